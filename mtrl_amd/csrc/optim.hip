// optim.hip -- clip_by_global_norm + Adam (+ Polyak target) + temperature update.
//
// Reference: OptimizerConfig.spawn (mtrl/config/optim.py:26-43) = optax.chain(
// clip_by_global_norm(max_grad_norm), adam(lr, eps=1e-5)); TrainState.apply_gradients
// (mtrl/rl/algorithms/utils.py:11-46); optax.incremental_update Polyak
// (mtsac.py:607-613); update_alpha (mtsac.py:713-731).
//
// Every network's parameters, gradients and moments live in ONE flat, 256-B aligned
// buffer each, so the whole optimizer is three streaming passes: sum of squares of
// the gradient (fixed grid -> deterministic partials), a one-block finalize, and the
// fused clip / Adam / Polyak / param-norm pass (7 x 4 B per parameter, +8 B for the
// target).  All reductions have a fixed shape, so results are run-to-run bitwise
// reproducible.
#include <algorithm>

#include "gemm_common.h"

namespace mtsac {

namespace {

__device__ inline float wsumf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ inline double wsumd(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// block-wide sum for 256 threads, result valid in thread 0
__device__ inline float block_sum256(float v) {
  __shared__ float s[4];
  v = wsumf(v);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0) r = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, long long n4,
                                                    float* __restrict__ partials) {
  float acc = 0.f;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 v = x4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = block_sum256(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void grad_norm_finalize_kernel(const float* __restrict__ partials, int nparts,
                                                                 const float* __restrict__ extra_sq,
                                                                 OptScalars* sc) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += (double)partials[i];
  acc = wsumd(acc);
  __shared__ double s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = (s[0] + s[1]) + (s[2] + s[3]);
    if (extra_sq) tot += (double)(*extra_sq);
    sc->gnorm = (float)sqrt(tot);
    sc->count += 1;  // optax safe_increment of the adam count
  }
}

__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partials, int nparts,
                                                           float* __restrict__ out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += (double)partials[i];
  acc = wsumd(acc);
  __shared__ double s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out = (float)((s[0] + s[1]) + (s[2] + s[3]));
}

// clip (t / ||g||) * max when !(||g|| < max); Adam: mu = (1-b1) g + b1 mu,
// nu = (1-b2) g^2 + b2 nu, mu_hat = mu / (1 - b1^k), nu_hat = nu / (1 - b2^k),
// p += -lr * mu_hat / (sqrt(nu_hat) + eps); then target = tau p + (1 - tau) target.
struct AdamConsts {
  bool clip;
  float gn, max_norm, bc1, bc2, omb1, omb2, neg_lr, omtau;
};

__device__ inline AdamConsts adam_consts(const AdamParams& a, float gnorm, int count, float max_norm) {
  AdamConsts k;
  k.clip = (max_norm >= 0.f) && !(gnorm < max_norm);
  k.gn = gnorm;
  k.max_norm = max_norm;
  k.bc1 = 1.0f - powf(a.b1, (float)count);
  k.bc2 = 1.0f - powf(a.b2, (float)count);
  k.omb1 = 1.0f - a.b1;
  k.omb2 = 1.0f - a.b2;
  k.neg_lr = -a.lr;
  k.omtau = 1.0f - a.tau;
  return k;
}

// the elementwise pass over float4 i = blk, blk + nblk, ... < n4 (tiled leaves skipped); returns
// this thread's |p_new|^2 over i >= norm_from4
// split2h: the exponents of the weights' planes this update writes (params, target), from the
// records' maxima of the values before the update (every block alike)
struct H2Scales {
  float sw, st;
};
__device__ inline H2Scales h2_scales(const AdamParams& a) {
  H2Scales s{1.f, 1.f};
  if (a.np != 2 || a.h2.wrec == nullptr) return s;
  const float bw = a.h2.wrec->amax[0] + a.h2.w_add;
  s.sw = exp2i(plane_exp(bw));
  if (a.h2.trec) s.st = exp2i(plane_exp(fmaxf(a.h2.trec->amax[0], bw)));
  return s;
}

template <bool POLYAK>
__device__ inline float adam_elems(const AdamParams& a, const AdamConsts& k, long long norm_from4, long long blk,
                                   long long nblk, float& pmx, float& tmx) {
  const long long n4 = a.n >> 2;
  float acc = 0.f;
  const H2Scales hs = h2_scales(a);
  float4* p4 = reinterpret_cast<float4*>(a.p);
  float4* m4 = reinterpret_cast<float4*>(a.m);
  float4* v4 = reinterpret_cast<float4*>(a.v);
  const float4* g4 = reinterpret_cast<const float4*>(a.g);
  float4* t4 = reinterpret_cast<float4*>(a.target);
  for (long long i = blk * 256 + threadIdx.x; i < n4; i += nblk * 256) {
    bool skip = false;
    for (int q = 0; q < a.nskip; ++q) skip |= i >= a.skip_b[q] && i < a.skip_e[q];
    if (skip) continue;  // a tiled leaf (adam_tiles)
    float4 p = p4[i];
    float* pp = &p.x;
    float sq = 0.f;
    if (a.refresh) {
#pragma unroll
      for (int c = 0; c < 4; ++c) sq += pp[c] * pp[c];
    } else {
      float4 g = g4[i], m = m4[i], v = v4[i];
      float* gp = &g.x;
      float* mp = &m.x;
      float* vp = &v.x;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float gk = gp[c];
        if (k.clip) gk = (gk / k.gn) * k.max_norm;
        mp[c] = k.omb1 * gk + a.b1 * mp[c];
        vp[c] = k.omb2 * (gk * gk) + a.b2 * vp[c];
        const float mh = mp[c] / k.bc1;
        const float vh = vp[c] / k.bc2;
        const float u = mh / (sqrtf(vh) + a.eps);
        pp[c] = pp[c] + u * k.neg_lr;
        sq += pp[c] * pp[c];
      }
      p4[i] = p;
      m4[i] = m;
      v4[i] = v;
    }
    if (a.whT != nullptr && i >= a.whT_b4 && i < a.whT_e4) {  // the head kernel, transposed per task
      const long long per = (long long)a.whT_W * a.whT_hd, f = 4 * (i - a.whT_b4);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const long long t = (f + c) / per, r = f + c - t * per;
        const int w = (int)(r / a.whT_hd), o = (int)(r - (long long)w * a.whT_hd);
        a.whT[(t * a.whT_hd + o) * a.whT_W + w] = pp[c];
      }
    }
    if (i >= norm_from4) acc += sq;  // |p|^2 of the replicated (trunk) range only
    pmx = fmaxf(pmx, fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fmaxf(fabsf(p.z), fabsf(p.w))));
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (POLYAK && t4 != nullptr) {
      t = t4[i];
      t.x = a.tau * p.x + k.omtau * t.x;
      t.y = a.tau * p.y + k.omtau * t.y;
      t.z = a.tau * p.z + k.omtau * t.z;
      t.w = a.tau * p.w + k.omtau * t.w;
      t4[i] = t;
      tmx = fmaxf(tmx, fmaxf(fmaxf(fabsf(t.x), fabsf(t.y)), fmaxf(fabsf(t.z), fabsf(t.w))));
    }
    for (int sg = 0; sg < a.nseg; ++sg) {  // split planes of the new values (next GEMMs' operands)
      const PlaneSeg& ps = a.seg[sg];
      const long long f = 4 * i - ps.begin;
      if (f < 0 || f >= ps.member_n * ps.members) continue;
      const long long e = f / ps.member_n, kk = f - e * ps.member_n;
      const float* src = ps.of_target ? &t.x : pp;
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      if (a.np == 2) {  // split2h planes
        const float sc = ps.of_target ? hs.st : hs.sw;
        f16x4 h2h, h2l;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          _Float16 x0, x1;
          split2h_dev(src[c], sc, x0, x1);
          h2h[c] = x0; h2l[c] = x1;
        }
        __bf16* dst = ps.planes + e * 3 * ps.ps + kk;
        *reinterpret_cast<f16x4*>(dst) = h2h;
        *reinterpret_cast<f16x4*>(dst + ps.ps) = h2l;
        continue;
      }
      bf16x4 h, mm, l;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const __bf16 hh = (__bf16)src[c];
        const float r1 = src[c] - (float)hh;
        const __bf16 m1 = (__bf16)r1;
        h[c] = hh;
        mm[c] = m1;
        l[c] = (__bf16)(r1 - (float)m1);
      }
      __bf16* dst = ps.planes + e * 3 * ps.ps + kk;
      *reinterpret_cast<bf16x4*>(dst) = h;
      if (a.np != 1) {
        *reinterpret_cast<bf16x4*>(dst + ps.ps) = mm;
        *reinterpret_cast<bf16x4*>(dst + 2 * ps.ps) = l;
      }
    }
  }
  return acc;
}

template <bool POLYAK>
__global__ __launch_bounds__(256) void adam_kernel(AdamParams a, float max_norm, long long norm_from4) {
  const OptScalars sc = *a.sc;
  const AdamConsts k = adam_consts(a, sc.gnorm, sc.count, max_norm);
  float pmx = 0.f, tmx = 0.f;
  float acc = adam_elems<POLYAK>(a, k, norm_from4, blockIdx.x, gridDim.x, pmx, tmx);
  acc = block_sum256(acc);
  if (threadIdx.x == 0) a.p_partials[blockIdx.x] = acc;
}

// 64 x 64 tiles of dense kernel leaves: thread t updates rows r0 + (t >> 4) + 16 j (j < 4), columns
// c0 + 4 (t & 15) .. + 3 (16-B loads, a row's 64 columns by 16 lanes); the new values go through
// LDS so the transposed planes leave as 2 x 16 B per lane (16 k of one output row).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// A tile's place and (no Polyak target) its four row groups' operands p, g, m, v, fetched ahead of the
// update: all of a tile's loads in flight together, the next tile's while this one's transposed planes
// are written, and a block's first tile's before the global norm is known.  Fetched row group by row
// group inside the update, each group's loads wait behind the previous group's stores (vmcnt counts
// stores).  Measured at C1 (`profiles/r5bl_*`): the actor's launch 15.3 -> 13.4 us; the critic's (five
// operands with the target, fetched the same way) 18.8 -> 22.2 us, so a Polyak network keeps the
// row-group loads.
struct TileFetch {
  int L, e, r0, c0;
  float4 p[4], g[4], m[4], v[4];
};

template <bool POLYAK>
__device__ inline void tile_fetch(const AdamParams& a, const TileParams& tp, int tile, TileFetch& F) {
  int L = 0;
  while (L + 1 < tp.n && tile >= tp.leaf[L + 1].tile_begin) ++L;
  const TileLeaf& lf = tp.leaf[L];
  int loc = tile - lf.tile_begin;
  const int per = lf.tiles_r * lf.tiles_c;
  F.L = L;
  F.e = loc / per;
  loc -= F.e * per;
  F.r0 = 64 * (loc / lf.tiles_c);
  F.c0 = 64 * (loc % lf.tiles_c);
  const long long base = lf.off + F.e * lf.ms;
  const int rr = threadIdx.x >> 4, c4 = 4 * (threadIdx.x & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = F.r0 + rr + 16 * j, c = F.c0 + c4;
    // outside the leaf: the leaf's first float4, loaded and never used (every load unconditional)
    const long long i4 = (r < lf.rows && c < lf.cols) ? (base + (long long)r * lf.cols + c) >> 2 : base >> 2;
    if constexpr (!POLYAK) {
      F.p[j] = reinterpret_cast<const float4*>(a.p)[i4];
      if (!a.refresh) {
        F.g[j] = reinterpret_cast<const float4*>(a.g)[i4];
        F.m[j] = reinterpret_cast<const float4*>(a.m)[i4];
        F.v[j] = reinterpret_cast<const float4*>(a.v)[i4];
      }
    }
  }
}

// 64 x 64 tile pass over tiles blk, blk + nblk, ... of tp (F holds tile blk's fetch when blk < total);
// returns this thread's |p_new|^2
template <bool POLYAK>
__device__ inline float adam_tiles(const AdamParams& a, const TileParams& tp, const AdamConsts& k, int blk, int nblk,
                                   float (*sp)[65], float (*stg)[65], float& pmx, float& tmx, TileFetch& F) {
  float acc = 0.f;
  const H2Scales hs = h2_scales(a);
  const int t = threadIdx.x, rr = t >> 4, c4 = 4 * (t & 15);
  for (int tile = blk; tile < tp.total; tile += nblk) {
    const int L = F.L, e = F.e, r0 = F.r0, c0 = F.c0;
    const TileLeaf& lf = tp.leaf[L];
    const long long base = lf.off + e * lf.ms;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + rr + 16 * j, c = c0 + c4;
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f), tv = p;
      if (r < lf.rows && c < lf.cols) {
        const long long i4 = (base + (long long)r * lf.cols + c) >> 2;
        p = POLYAK ? reinterpret_cast<float4*>(a.p)[i4] : F.p[j];
        float* pp = &p.x;
        if (a.refresh) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc += pp[q] * pp[q];
            pmx = fmaxf(pmx, fabsf(pp[q]));
          }
        } else {
          float4 g = POLYAK ? reinterpret_cast<const float4*>(a.g)[i4] : F.g[j];
          float4 m = POLYAK ? reinterpret_cast<float4*>(a.m)[i4] : F.m[j];
          float4 v = POLYAK ? reinterpret_cast<float4*>(a.v)[i4] : F.v[j];
          float* gp = &g.x;
          float* mp = &m.x;
          float* vp = &v.x;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float gk = gp[q];
            if (k.clip) gk = (gk / k.gn) * k.max_norm;
            mp[q] = k.omb1 * gk + a.b1 * mp[q];
            vp[q] = k.omb2 * (gk * gk) + a.b2 * vp[q];
            const float mh = mp[q] / k.bc1;
            const float vh = vp[q] / k.bc2;
            const float u = mh / (sqrtf(vh) + a.eps);
            pp[q] = pp[q] + u * k.neg_lr;
            acc += pp[q] * pp[q];
            pmx = fmaxf(pmx, fabsf(pp[q]));
          }
          reinterpret_cast<float4*>(a.p)[i4] = p;
          reinterpret_cast<float4*>(a.m)[i4] = m;
          reinterpret_cast<float4*>(a.v)[i4] = v;
        }
        if (POLYAK) {
          tv = reinterpret_cast<float4*>(a.target)[i4];
          tv.x = a.tau * p.x + k.omtau * tv.x;
          tv.y = a.tau * p.y + k.omtau * tv.y;
          tv.z = a.tau * p.z + k.omtau * tv.z;
          tv.w = a.tau * p.w + k.omtau * tv.w;
          reinterpret_cast<float4*>(a.target)[i4] = tv;
          tmx = fmaxf(tmx, fmaxf(fmaxf(fabsf(tv.x), fabsf(tv.y)), fmaxf(fabsf(tv.z), fabsf(tv.w))));
        }
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          __bf16* np_ = lf.nat[w];
          if (np_ == nullptr || (w == 1 && !POLYAK)) continue;
          const float* src = w ? &tv.x : &p.x;
          if (a.np == 2) {  // split2h planes
            f16x4 h2h, h2l;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              _Float16 x0, x1;
              split2h_dev(src[q], w ? hs.st : hs.sw, x0, x1);
              h2h[q] = x0; h2l[q] = x1;
            }
            __bf16* dst = np_ + e * 3 * lf.nat_ps + (lf.frag ? frag_off(r, c, lf.nat_ld) : (long long)r * lf.nat_ld + c);
            *reinterpret_cast<f16x4*>(dst) = h2h;
            *reinterpret_cast<f16x4*>(dst + lf.nat_ps) = h2l;
            continue;
          }
          bf16x4_t h, mm, l;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            __bf16 x0, x1, x2;
            split3_dev(src[q], x0, x1, x2);
            h[q] = x0; mm[q] = x1; l[q] = x2;
          }
          __bf16* dst = np_ + e * 3 * lf.nat_ps + (lf.frag ? frag_off(r, c, lf.nat_ld) : (long long)r * lf.nat_ld + c);
          *reinterpret_cast<bf16x4_t*>(dst) = h;
          if (a.np != 1) {
            *reinterpret_cast<bf16x4_t*>(dst + lf.nat_ps) = mm;
            *reinterpret_cast<bf16x4_t*>(dst + 2 * lf.nat_ps) = l;
          }
        }
      }
      const int lr_ = rr + 16 * j;
      sp[lr_][c4] = p.x; sp[lr_][c4 + 1] = p.y; sp[lr_][c4 + 2] = p.z; sp[lr_][c4 + 3] = p.w;
      if (POLYAK) {
        stg[lr_][c4] = tv.x; stg[lr_][c4 + 1] = tv.y; stg[lr_][c4 + 2] = tv.z; stg[lr_][c4 + 3] = tv.w;
      }
    }
    if (tile + nblk < tp.total) tile_fetch<POLYAK>(a, tp, tile + nblk, F);  // F's registers are free now
    __syncthreads();
    {  // transposed planes: output row o (a column of the leaf), k = r0 + 16 (t & 3) .. + 15
      const int oc = t >> 2, kq = 16 * (t & 3);
      const int o = c0 + oc, kk = r0 + kq;
      if (o < lf.cols && kk < lf.tr_ld) {
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          __bf16* tp_ = lf.tr[w];
          if (tp_ == nullptr || (w == 1 && !POLYAK)) continue;
          // the two 8-k halves: adjacent, or (fragment layout) 16 lanes = 128 elements apart
          __bf16* dst = tp_ + e * 3 * lf.tr_ps + (lf.frag ? frag_off(o, kk, lf.tr_ld) : (long long)o * lf.tr_ld + kk);
          const int hs8 = lf.frag ? 128 : 8;
          if (a.np == 2) {  // split2h planes
            f16x8 h2h[2], h2l[2];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              const float x = w ? stg[POLYAK ? kq + q : 0][oc] : sp[kq + q][oc];
              _Float16 x0, x1;
              split2h_dev(x, w ? hs.st : hs.sw, x0, x1);
              h2h[q >> 3][q & 7] = x0; h2l[q >> 3][q & 7] = x1;
            }
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              if (kk + 8 * hh >= lf.tr_ld) break;
              *reinterpret_cast<f16x8*>(dst + hs8 * hh) = h2h[hh];
              *reinterpret_cast<f16x8*>(dst + lf.tr_ps + hs8 * hh) = h2l[hh];
            }
            continue;
          }
          bf16x8 h[2], mm[2], l[2];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const float x = w ? stg[POLYAK ? kq + q : 0][oc] : sp[kq + q][oc];
            __bf16 x0, x1, x2;
            split3_dev(x, x0, x1, x2);
            h[q >> 3][q & 7] = x0; mm[q >> 3][q & 7] = x1; l[q >> 3][q & 7] = x2;
          }
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            if (kk + 8 * hh >= lf.tr_ld) break;
            *reinterpret_cast<bf16x8*>(dst + hs8 * hh) = h[hh];
            if (a.np != 1) {
              *reinterpret_cast<bf16x8*>(dst + lf.tr_ps + hs8 * hh) = mm[hh];
              *reinterpret_cast<bf16x8*>(dst + 2 * lf.tr_ps + hs8 * hh) = l[hh];
            }
          }
        }
      }
    }
    __syncthreads();
  }
  return acc;
}

template <bool POLYAK>
__global__ __launch_bounds__(256) void adam_tiles_kernel(AdamParams a, TileParams tp, float max_norm) {
  __shared__ float sp[64][65];
  __shared__ float stg[POLYAK ? 64 : 1][65];
  TileFetch F;
  if ((int)blockIdx.x < tp.total) tile_fetch<POLYAK>(a, tp, blockIdx.x, F);
  const OptScalars sc = *a.sc;
  const AdamConsts k = adam_consts(a, sc.gnorm, sc.count, max_norm);
  float pmx = 0.f, tmx = 0.f;
  float acc = adam_tiles<POLYAK>(a, tp, k, blockIdx.x, gridDim.x, sp, stg, pmx, tmx, F);
  acc = block_sum256(acc);
  if (threadIdx.x == 0) a.p_partials[blockIdx.x] = acc;
}

// One launch for a whole network's optimizer step (engine.cpp optimize): every block recomputes the
// global gradient norm from the sum-of-squares partials in the same fixed order (so every block, and
// every rank's replicated trunk, sees the same clip factor), then blocks [0, bh) run the heads'
// elementwise update, [bh, bh + bt) the trunk's elementwise leaves, the rest its 64 x 64 kernel
// tiles.  |p_new|^2 partials: heads to f.ph[blk], trunk to f.pt[blk - bh].
template <bool POLYAK>
__global__ __launch_bounds__(256) void adam_fused_kernel(AdamParams ah, AdamParams at, TileParams tp, FusedOpt f) {
  __shared__ float sp[64][65];
  __shared__ float stg[POLYAK ? 64 : 1][65];
  __shared__ double red[4];
  __shared__ float gsh;
  // the global norm: the trunk's and (unsharded) the heads' |g|^2 partials, both summed by the whole
  // block in a fixed order (the heads' were summed by one thread, a serial chain of up to 256 loads that
  // every block of the launch waited for)
  __shared__ double hred[4];
  // a tile block's first tile is fetched before the norm's partials: both round trips overlap
  const int b = blockIdx.x, tb = b - f.bh - f.bt;
  TileFetch F;
  if (tb >= 0 && tb < tp.total) tile_fetch<POLYAK>(at, tp, tb, F);
  double acc = 0.0, hacc = 0.0;
  for (int i = threadIdx.x; i < f.ng; i += 256) acc += (double)f.gparts[i];
  if (!f.head_sq)
    for (int i = threadIdx.x; i < f.nh; i += 256) hacc += (double)f.hparts[i];
  acc = wsumd(acc);
  hacc = wsumd(hacc);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = acc;
    hred[threadIdx.x >> 6] = hacc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = (red[0] + red[1]) + (red[2] + red[3]);
    const float head = f.head_sq ? *f.head_sq : (float)((hred[0] + hred[1]) + (hred[2] + hred[3]));
    gsh = (float)sqrt(tot + (double)head);
  }
  __syncthreads();
  const float gn = gsh;
  const int count = ah.sc->count;  // incremented by the sum-of-squares launch
  float pa = 0.f, pmx = 0.f, tmx = 0.f;
  if (b < f.bh) {
    pa = adam_elems<POLYAK>(ah, adam_consts(ah, gn, count, f.max_norm), 0, b, f.bh, pmx, tmx);
  } else if (b < f.bh + f.bt) {
    pa = adam_elems<POLYAK>(at, adam_consts(at, gn, count, f.max_norm), 0, b - f.bh, f.bt, pmx, tmx);
  } else {
    pa = adam_tiles<POLYAK>(at, tp, adam_consts(at, gn, count, f.max_norm), tb, f.btile, sp, stg, pmx, tmx, F);
  }
  pa = block_sum256(pa);
  if (threadIdx.x == 0) {
    if (b < f.bh) f.ph[b] = pa;
    else f.pt[b - f.bh] = pa;
    if (b == 0) ah.sc->gnorm = gn;
  }
  if (at.np == 2 && at.h2.wrec) {  // split2h: the block's max |p_new| (|t_new|), reduced by step_finish
    __shared__ float mscr[16];
    pmx = block_max_val(pmx, mscr);
    tmx = block_max_val(tmx, mscr);
    if (threadIdx.x == 0) {
      at.h2.wparts[b] = pmx;
      if (at.h2.tparts) at.h2.tparts[b] = tmx;
      if (b == 0) {  // the exponents the planes of this update carry (every block derived them alike)
        const float bw = at.h2.wrec->amax[0] + at.h2.w_add;
        at.h2.wrec->e = plane_exp(bw);
        if (at.h2.trec) at.h2.trec->e = plane_exp(fmaxf(at.h2.trec->amax[0], bw));
      }
    }
  }
}

// the sharded optimizer's |g|^2: per block over this rank's shard ranges; block 0 bumps the Adam count
__global__ __launch_bounds__(256) void shard_sumsq_kernel(const float* __restrict__ g, ShardRanges r,
                                                          float* __restrict__ part, OptScalars* sc) {
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float acc = 0.f;
  for (int q = 0; q < r.n; ++q)
    for (long long i = r.b[q] + (long long)blockIdx.x * 256 + threadIdx.x; i < r.e[q]; i += (long long)gridDim.x * 256) {
      const float4 v = g4[i];
      acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  acc = block_sum256(acc);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = acc;
    if (blockIdx.x == 0) sc->count += 1;
  }
}

// *out += sum(partials) in a fixed order (one block, double accumulation)
__global__ __launch_bounds__(256) void sum_partials_add_kernel(const float* __restrict__ partials, int nparts,
                                                               float* __restrict__ out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += (double)partials[i];
  acc = wsumd(acc);
  __shared__ double s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out = (float)((double)*out + ((s[0] + s[1]) + (s[2] + s[3])));
}

// |g|^2 partials of a network: blocks [0, gh) over the heads' range, [gh, gh + gt) over the trunk's;
// block 0 bumps the Adam step count (optax's count, read by adam_fused_kernel)
__global__ __launch_bounds__(256) void sumsq2_kernel(const float* __restrict__ h, long long nh4, int gh,
                                                     const float* __restrict__ t, long long nt4, float* __restrict__ hp,
                                                     float* __restrict__ tp, OptScalars* sc) {
  const bool head = (int)blockIdx.x < gh;
  const float4* x4 = reinterpret_cast<const float4*>(head ? h : t);
  const long long n4 = head ? nh4 : nt4;
  const long long b = head ? blockIdx.x : blockIdx.x - gh, nb = head ? gh : gridDim.x - gh;
  float acc = 0.f;
  for (long long i = b * 256 + threadIdx.x; i < n4; i += nb * 256) {
    const float4 v = x4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = block_sum256(acc);
  if (threadIdx.x == 0) {
    if (head) hp[b] = acc;
    else tp[b] = acc;
    if (blockIdx.x == 0) sc->count += 1;
  }
}

struct RowPtrs {
  const float* p[4];
};

__global__ __launch_bounds__(1024) void reduce_rows_kernel(RowPtrs in, int n_in, int B, float* __restrict__ out) {
  __shared__ double s[16];
  for (int k = 0; k < n_in; ++k) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < B; i += 1024) acc += (double)in.p[k][i];
    acc = wsumd(acc);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int w = 0; w < 16; ++w) t += s[w];
      out[k] = (float)t;
    }
    __syncthreads();
  }
}

// temperature gradient: d/dlogalpha_t mean_b(-(x_b . logalpha)(logpi_b + H))
//   = -(1/B) sum_{b in t}(logpi_b + H)    (x one-hot, validated by the gather)
// zero outside this shard's tasks; the loss term of each task goes to task_loss[t]
// one block of 16 waves, wave w over the global tasks w, w + 16, ...; after the barrier wave 0
// sums the per-task loss terms in task order
// the per-task sums of waves [0, nw): wave w takes global tasks w, w + nw, ...
// Four tasks per wave at a time, every load unconditional (clamped index, value selected after): a
// load under a branch was waited for one task at a time (three dependent round trips per task).
__device__ void alpha_tasks(const AlphaParams& a, int wave, int nw) {
  const int lane = threadIdx.x & 63;
  constexpr int U = 4;
  for (int tg0 = wave; tg0 < a.T_glob; tg0 += U * nw) {
    int tl[U], n[U];
    bool ok[U];
    float la[U];  // log_alpha of the tasks, loaded beside the counts (read after the sums)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = tg0 + u * nw - a.task_begin;
      ok[u] = tg0 + u * nw < a.T_glob && t >= 0 && t < a.T_l;
      tl[u] = ok[u] ? t : 0;
      const int c = a.counts[tl[u]];
      n[u] = ok[u] ? c : 0;
      la[u] = a.log_alpha[min(tg0 + u * nw, a.T_glob - 1)];
    }
    int nmax = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) nmax = max(nmax, n[u]);  // wave-uniform
    float s[U] = {0.f, 0.f, 0.f, 0.f};
    // two 64-row chunks a pass (all their loads in flight together), added chunk by chunk in row order
    // as one chunk a pass did; rows past a task's count add +0 (s is never -0, so that is exact)
    for (int j0 = 0; j0 < nmax; j0 += 128) {
      int r[2][U];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = j0 + 64 * h + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rr = a.rows[(long long)tl[u] * a.max_rows + min(j, a.max_rows - 1)];
          r[h][u] = j < n[u] ? rr : 0;
        }
      }
      float lp[2][U];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < U; ++u) lp[h][u] = a.logpi[r[h][u]];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = j0 + 64 * h + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) s[u] += j < n[u] ? lp[h][u] + a.target_entropy : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = wsumf(s[u]);
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int tg = tg0 + u * nw;
        if (tg >= a.T_glob) continue;
        a.grad[tg] = ok[u] ? -s[u] / (float)a.B_glob : 0.f;
        a.task_loss[tg] = ok[u] ? -la[u] * s[u] : 0.f;
      }
    }
  }
}

__device__ void alpha_grad_block(const AlphaParams& a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  alpha_tasks(a, wave, 16);
  __syncthreads();
  if (wave == 0) {
    float s = 0.f;
    for (int t = lane; t < a.T_glob; t += 64) s += a.task_loss[t];
    s = wsumf(s);
    if (lane == 0) *a.loss_part = s;
  }
}

__global__ __launch_bounds__(1024) void alpha_grad_kernel(AlphaParams a) { alpha_grad_block(a); }

// temperature Adam (optax clip_by_global_norm + adam over log_alpha); one wave.  Returns the alpha log
// sum(exp(log_alpha_new)) (wave-uniform).  Up to 64 tasks: one task a lane, every operand loaded at
// once (the strided loops' loads were waited for loop by loop); the same sums, so the same bits.
__device__ float alpha_adam_wave(const AlphaParams& a, float lr, float b1, float b2, float eps, float max_norm) {
  const int lane = threadIdx.x & 63;
  const int count = a.sc->count + 1;
  const float bc1 = 1.0f - powf(b1, (float)count), bc2 = 1.0f - powf(b2, (float)count);
  float gn, es = 0.f;
  bool clip;
  if (a.T_glob <= 64) {
    const int i = min(lane, a.T_glob - 1);
    const bool in = lane < a.T_glob;
    const float g0 = a.grad[i], m0 = a.m[i], v0 = a.v[i], p0 = a.log_alpha[i];
    gn = sqrtf(wsumf(in ? 0.f + g0 * g0 : 0.f));
    clip = (max_norm >= 0.f) && !(gn < max_norm);
    float g = g0;
    if (clip) g = (g / gn) * max_norm;
    const float m = (1.0f - b1) * g + b1 * m0;
    const float v = (1.0f - b2) * (g * g) + b2 * v0;
    const float u = (m / bc1) / (sqrtf(v / bc2) + eps);
    const float p = p0 + u * (-lr);
    if (in) {
      a.m[i] = m;
      a.v[i] = v;
      a.log_alpha[i] = p;
    }
    es = in ? 0.f + expf(p) : 0.f;
  } else {
    float sq = 0.f;
    for (int i = lane; i < a.T_glob; i += 64) sq += a.grad[i] * a.grad[i];
    gn = sqrtf(wsumf(sq));
    clip = (max_norm >= 0.f) && !(gn < max_norm);
    for (int i = lane; i < a.T_glob; i += 64) {
      float g = a.grad[i];
      if (clip) g = (g / gn) * max_norm;
      const float m = (1.0f - b1) * g + b1 * a.m[i];
      const float v = (1.0f - b2) * (g * g) + b2 * a.v[i];
      a.m[i] = m;
      a.v[i] = v;
      const float u = (m / bc1) / (sqrtf(v / bc2) + eps);
      const float p = a.log_alpha[i] + u * (-lr);
      a.log_alpha[i] = p;
      es += expf(p);
    }
  }
  es = wsumf(es);
  if (lane == 0) {
    a.sc->count = count;
    a.sc->gnorm = gn;
    a.sc->pnorm = es;  // alpha log: sum(exp(log_alpha))  (mtsac.py:730)
  }
  return es;
}

// wave 0: the logs.  Values this launch produced come in as arguments (the alpha log sum, and when the
// log's source is this launch's output, the row sums, the alpha loss and the parameter norms); the rest
// are loaded (sharded runs reduce some elsewhere).  One store -> load round trip less per value.
struct LogLocal {
  float alpha_sum;
  float rows[3];        // valid where f.rows[k]
  float alpha_loss;     // valid with f.alpha_grad
  float pnorm[2];       // critic, actor
};

// the step's scalar tail in one block, its independent reductions side by side before ONE barrier:
// waves 0-7 the temperature gradient's per-task sums (unsharded), waves 8-15 the loss row sums (three
// [B] vectors, unsharded) and both networks' post-update |p| partials (waves 8-11 critic, 12-15
// actor); then wave 0 finishes everything in fixed orders (alpha loss, row sums, norms), the
// temperature Adam, the logs and the step counter.
__global__ __launch_bounds__(1024) void step_finish_kernel(StepFinish f) {
  __shared__ double s[48];  // [8 k + w] row sum k of wave 8 + w; [24 + 2 w + {0,1}] trunk / head |p|^2 of wave 8 + w
  __shared__ float wm[3][8][2];  // split2h: [job][wave 8 + w][heads, trunk] partial weight maxima
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // wave 0's inputs from earlier launches (the gradient norms, the step counter), loaded up front
  unsigned long long cnt = 0;
  float cgn = 0.f, agn = 0.f;
  if (wave == 0) {
    cnt = *f.counter;
    cgn = f.logs.critic->gnorm;
    agn = f.logs.actor->gnorm;
  }
  if (wave < 8) {
    if (f.alpha_grad) alpha_tasks(f.alpha, wave, 8);
  } else {
    {  // split2h: the optimizer's per-block weight maxima, strided over waves 8-15 (loads outside any
       // branch: a load under a condition was waited for one iteration at a time)
      const int u = threadIdx.x - 512, wl = wave - 8;
      for (int j = 0; j < f.nwmax; ++j) {
        const WeightMaxJob& w = f.wmax[j];
        float mh = 0.f, mt = 0.f;
        for (int i = u; i < w.n; i += 512) {
          const float v = w.parts[i];
          mh = i < w.nh ? fmaxf(mh, v) : mh;
          mt = i < w.nh ? mt : fmaxf(mt, v);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          mh = fmaxf(mh, __shfl_xor(mh, o));
          mt = fmaxf(mt, __shfl_xor(mt, o));
        }
        if (lane == 0) {
          wm[j][wl][0] = mh;
          wm[j][wl][1] = mt;
        }
      }
    }
    const int u = threadIdx.x - 512, wl = wave - 8;
    double r[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (f.rows[k])
        for (int i = u; i < f.B; i += 512) r[k] += (double)f.rows[k][i];
    const int w = u >> 8, v = u & 255;  // network: waves 8-11 critic, 12-15 actor
    double t = 0.0, h = 0.0;
    for (int i = v; i < f.pn.nt[w]; i += 256) t += (double)f.pn.pt[w][i];
    for (int i = v; i < f.pn.nh[w]; i += 256) h += (double)f.pn.ph[w][i];
#pragma unroll
    for (int k = 0; k < 3; ++k) r[k] = wsumd(r[k]);
    t = wsumd(t);
    h = wsumd(h);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) s[8 * k + wl] = r[k];
      s[24 + 2 * wl] = t;
      s[24 + 2 * wl + 1] = h;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  const AlphaParams& a = f.alpha;
  LogLocal loc{};
  if (f.alpha_grad) {  // the alpha loss: the per-task terms in task order
    float sl = 0.f;
    for (int t = lane; t < a.T_glob; t += 64) sl += a.task_loss[t];
    sl = wsumf(sl);
    loc.alpha_loss = sl;
    if (lane == 0) *a.loss_part = sl;
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (!f.rows[k]) continue;
      double t = 0.0;
      for (int w = 0; w < 8; ++w) t += s[8 * k + w];
      loc.rows[k] = (float)t;
      *f.row_out[k] = loc.rows[k];
    }
    for (int n = 0; n < 2; ++n) {
      double tt = 0.0, hh = 0.0;
      for (int w = 4 * n; w < 4 * n + 4; ++w) {
        tt += s[24 + 2 * w];
        hh += s[24 + 2 * w + 1];
      }
      const float hs = f.head_sq ? f.head_sq[n] : (float)hh;
      loc.pnorm[n] = sqrtf((float)tt + hs);
      f.pn.sc[n]->pnorm = loc.pnorm[n];
    }
  }
  loc.alpha_sum = alpha_adam_wave(f.alpha, f.lr, f.b1, f.b2, f.eps, f.max_norm);
  // the logs: a value this launch produced is taken from registers when the log's source is where it
  // was stored (the engine's layout); anything else is loaded after a fence
  const LogParams& p = f.logs;
  const bool own_c0 = f.rows[0] && p.critic_sums == f.row_out[0];
  const bool own_c1 = f.rows[1] && p.critic_sums + 1 == f.row_out[1];
  const bool own_a = f.rows[2] && p.actor_sums == f.row_out[2];
  const bool own_al = f.alpha_grad && p.alpha_loss_sum == a.loss_part;
  const bool own_pn = f.pn.sc[0] == p.critic && f.pn.sc[1] == p.actor;
  const bool own_ls = p.log_alpha == a.log_alpha && p.T_glob == a.T_glob;
  if (!(own_c0 && own_c1 && own_a && own_al && own_pn && own_ls)) __threadfence_block();
  float ls = loc.alpha_sum;
  if (!own_ls) {  // wave 0: the alpha log summed lane-strided (the loads in flight together)
    float s2 = 0.f;
    for (int i = lane; i < p.T_glob; i += 64) s2 += expf(p.log_alpha[i]);
    ls = wsumf(s2);
  }
  if (lane == 0) {
    p.logs[0] = (own_c1 ? loc.rows[1] : p.critic_sums[1]) * p.inv_critic;  // losses/qf_values
    p.logs[1] = (own_c0 ? loc.rows[0] : p.critic_sums[0]) * p.inv_critic;  // losses/qf_loss
    p.logs[2] = cgn;                                                          // metrics/critic_grad_magnitude
    p.logs[3] = own_pn ? loc.pnorm[0] : p.critic->pnorm;                      // metrics/critic_params_norm
    p.logs[4] = (own_a ? loc.rows[2] : p.actor_sums[0]) * p.inv_actor;      // losses/actor_loss
    p.logs[5] = agn;                                                          // metrics/actor_grad_magnitude
    p.logs[6] = own_pn ? loc.pnorm[1] : p.actor->pnorm;                       // metrics/actor_params_norm
    p.logs[7] = 0.0f;  // metrics/explore_loss (explore=False, mtsac.py:277)
    p.logs[8] = (own_al ? loc.alpha_loss : *p.alpha_loss_sum) * p.inv_b;      // losses/alpha_loss
    p.logs[9] = ls;                                                           // alpha
    *f.counter = cnt + 1ull;
  }
  // split2h: the optimizer's per-block weight maxima into the weight records (the next update's bound)
  for (int j = 0; j < f.nwmax; ++j) {
    const WeightMaxJob& w = f.wmax[j];
    float mh = 0.f, mt = 0.f;
    for (int q = 0; q < 8; ++q) {
      mh = fmaxf(mh, wm[j][q][0]);
      mt = fmaxf(mt, wm[j][q][1]);
    }
    if (lane == 0) {
      if (w.nh < 0) {
        w.rec->amax[0] = mt;  // a target: heads and trunk together (a looser, valid bound)
      } else {
        w.rec->amax[0] = mt;
        w.rec->amax[1] = mh;
      }
    }
  }
}

}  // namespace

// split2h, weights set from outside (set_params): the record's maxima (trunk -> amax[0], heads ->
// amax[1]) and the planes' exponent from the exact trunk maximum; one block (a rare call)
__global__ __launch_bounds__(1024) void weights_record_kernel(const float* __restrict__ p, long long trunk_off,
                                                             long long n_flat, PlaneRec* rec) {
  __shared__ float mscr[16];
  float mh = 0.f, mt = 0.f;
  for (long long i = threadIdx.x; i < n_flat; i += 1024) {
    const float v = fabsf(p[i]);
    if (i < trunk_off) mh = fmaxf(mh, v);
    else mt = fmaxf(mt, v);
  }
  mh = block_max_val(mh, mscr);
  mt = block_max_val(mt, mscr);
  if (threadIdx.x == 0) {
    rec->amax[0] = mt;
    rec->amax[1] = mh;
    rec->e = plane_exp(mt);
  }
}

void weights_record(const float* p, long long trunk_off, long long n_flat, PlaneRec* rec, hipStream_t st) {
  hipLaunchKernelGGL(weights_record_kernel, dim3(1), dim3(1024), 0, st, p, trunk_off, n_flat, rec);
}

void reduce_rows(const float* const* ins, int n_in, int B, float* out, hipStream_t st) {
  RowPtrs r{};
  for (int i = 0; i < n_in && i < 4; ++i) r.p[i] = ins[i];
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(1), dim3(1024), 0, st, r, n_in, B, out);
}

int sumsq_partials(const float* x, long long n, float* partials, int max_blocks, hipStream_t st) {
  const long long n4 = n >> 2;
  long long g = (n4 + 255) / 256;
  if (g > max_blocks) g = max_blocks;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)g), dim3(256), 0, st, x, n4, partials);
  return (int)g;
}

void grad_norm_finalize(const float* partials, int nparts, const float* extra_sq, float max_norm, OptScalars* sc,
                        hipStream_t st) {
  (void)max_norm;
  hipLaunchKernelGGL(grad_norm_finalize_kernel, dim3(1), dim3(256), 0, st, partials, nparts, extra_sq, sc);
}

int adam_update(const AdamParams& a, float max_norm, long long norm_from, int max_blocks, hipStream_t st) {
  const long long n4 = a.n >> 2;
  long long g = (n4 + 255) / 256;
  if (g > max_blocks) g = max_blocks;
  if (g < 1) g = 1;
  if (a.target)
    hipLaunchKernelGGL(adam_kernel<true>, dim3((unsigned)g), dim3(256), 0, st, a, max_norm, norm_from >> 2);
  else
    hipLaunchKernelGGL(adam_kernel<false>, dim3((unsigned)g), dim3(256), 0, st, a, max_norm, norm_from >> 2);
  return (int)g;
}

int adam_update_tiles(const AdamParams& a, const TileParams& tp, float max_norm, int max_blocks, hipStream_t st) {
  int g = std::min(tp.total, max_blocks);
  if (g < 1) g = 1;
  if (a.target)
    hipLaunchKernelGGL(adam_tiles_kernel<true>, dim3((unsigned)g), dim3(256), 0, st, a, tp, max_norm);
  else
    hipLaunchKernelGGL(adam_tiles_kernel<false>, dim3((unsigned)g), dim3(256), 0, st, a, tp, max_norm);
  return g;
}

__global__ void pnorm_finalize_kernel(const float* __restrict__ trunk_sq, const float* __restrict__ head_sq,
                                      OptScalars* s0, OptScalars* s1) {
  s0->pnorm = sqrtf(trunk_sq[0] + head_sq[0]);
  s1->pnorm = sqrtf(trunk_sq[1] + head_sq[1]);
}

void pnorm_finalize(const float* trunk_sq, const float* head_sq, OptScalars* s0, OptScalars* s1, hipStream_t st) {
  hipLaunchKernelGGL(pnorm_finalize_kernel, dim3(1), dim3(1), 0, st, trunk_sq, head_sq, s0, s1);
}


int sumsq2(const float* h, long long nh, const float* t, long long nt, float* hparts, float* tparts, OptScalars* sc,
           int* gh_out, hipStream_t st) {
  const long long nh4 = nh >> 2, nt4 = nt >> 2;
  const int gh = h ? (int)std::max<long long>(1, std::min<long long>(FUSED_HEAD_PARTS, (nh4 + 255) / 256)) : 0;
  const int gt = (int)std::max<long long>(1, std::min<long long>(1024, (nt4 + 255) / 256));
  hipLaunchKernelGGL(sumsq2_kernel, dim3((unsigned)(gh + gt)), dim3(256), 0, st, h, nh4, gh, t, nt4, hparts, tparts, sc);
  *gh_out = gh;
  return gt;
}

void adam_fused(const AdamParams& ah, const AdamParams& at, const TileParams& tp, FusedOpt& f, hipStream_t st) {
  f.bh = (int)std::max<long long>(1, std::min<long long>(FUSED_HEAD_PARTS, ((ah.n >> 2) + 255) / 256));
  f.bt = (int)std::max<long long>(1, std::min<long long>(1024, ((at.n >> 2) + 255) / 256));
  f.btile = std::min(tp.total, 1024);
  const dim3 grid((unsigned)(f.bh + f.bt + f.btile));
  if (at.target)
    hipLaunchKernelGGL(adam_fused_kernel<true>, grid, dim3(256), 0, st, ah, at, tp, f);
  else
    hipLaunchKernelGGL(adam_fused_kernel<false>, grid, dim3(256), 0, st, ah, at, tp, f);
}

void shard_sumsq_add(const float* g, const ShardRanges& r, float* partials, float* out, OptScalars* sc,
                     hipStream_t st) {
  long long n4 = 0;
  for (int q = 0; q < r.n; ++q) n4 += r.e[q] - r.b[q];
  const int G = (int)std::max<long long>(1, std::min<long long>(256, (n4 + 1023) / 1024));
  hipLaunchKernelGGL(shard_sumsq_kernel, dim3(G), dim3(256), 0, st, g, r, partials, sc);
  hipLaunchKernelGGL(sum_partials_add_kernel, dim3(1), dim3(256), 0, st, partials, G, out);
}

void sum_partials(const float* partials, int nparts, float* out, hipStream_t st) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, st, partials, nparts, out);
}

void alpha_grad(const AlphaParams& a, hipStream_t st) {
  hipLaunchKernelGGL(alpha_grad_kernel, dim3(1), dim3(1024), 0, st, a);
}

void step_finish(const StepFinish& f, hipStream_t st) {
  hipLaunchKernelGGL(step_finish_kernel, dim3(1), dim3(1024), 0, st, f);
}

}  // namespace mtsac
