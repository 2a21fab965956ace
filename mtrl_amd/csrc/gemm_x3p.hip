// gemm_x3p.hip -- fp32-accurate GEMM on PRE-SPLIT bf16 planes (gfx950).
//
// Operands arrive as three bf16 planes each (x = x_h + x_m + x_l exactly, see gemm_x3.hip), so
// the main loop has no VALU at all:
//   C[M][N] = sum_k A(m, k) B(n, k), A given either row-major [3][M][lda] (k contiguous) or
//   k-major [3][K][lda] (m contiguous), B likewise with N.  K is a multiple of 32; the planes
//   of row-major operands carry zeros in k >= K up to the next multiple of 32.
//   * global -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane) into a ring of
//     STAGES K-steps, counted vmcnt + one raw s_barrier per 32-deep K-step;
//   * row-major image [rows][4 x 16 B] per plane, chunk XOR (row >> 2) & 3, read with one
//     ds_read_b128 per lane; k-major image [32 k][rows] per plane, chunk XOR 4 * (k & 3),
//     read with two ds_read_b64_tr_b16 per lane (hardware transpose).  The swizzles are
//     applied on the SOURCE address (the DMA writes lane-linearly); both reads are
//     bank-conflict free;
//   * 6 x v_mfma_f32_32x32x16_bf16 per 32x32 tile and 16-deep k-slice (m*m, h*l, l*h, h*m,
//     m*h, h*h; small terms first), fp32 accumulation;
//   * optional split-K: slices of K write dense partial slabs, reduced in slice order.
// Epilogue: fp32 C with bias+ReLU / ReLU-mask / plain, and optionally the split planes of C
// (natural layout) for the next GEMM.
#include <algorithm>

#include "gemm_x3p_impl.h"

namespace mtsac {

using x3pk::BK;

namespace {

// fp32 [rows][ld] -> planes.  TRANS: out[q][col][row] (k = row contiguous), else out[q][row][col].
// 64x64 tiles staged through LDS so both the fp32 reads and the bf16 writes are coalesced.
template <bool TRANS>
__global__ __launch_bounds__(256) void split_kernel(SplitParams s) {
  __shared__ float tile[64][65];
  const int z = blockIdx.z;
  const float* __restrict__ x = s.x + z * s.sx;
  __bf16* __restrict__ out = s.out + z * s.so;
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int t = threadIdx.x;
  // load 64 x 64 (zero outside [rows, cols)): thread t reads col c0 + (t & 63), rows r0 + (t>>6) + 4i
  for (int i = 0; i < 16; ++i) {
    const int r = (t >> 6) + 4 * i, c = t & 63;
    const int gr = r0 + r, gc = c0 + c;
    tile[r][c] = (gr < s.rows && gc < s.cols) ? x[(long long)gr * s.ldx + gc] : 0.f;
  }
  __syncthreads();
  for (int i = 0; i < 16; ++i) {
    int a = (t >> 6) + 4 * i, b = t & 63;  // output row a, output col b (within the tile)
    float v;
    long long o;
    if (TRANS) {  // output row = source col, output col = source row
      v = tile[b][a];
      const int orow = c0 + a, ocol = r0 + b;
      if (orow >= s.out_rows || ocol >= s.out_cols) continue;
      o = s.frag ? frag_off(orow, ocol, s.ldo) : (long long)orow * s.ldo + ocol;
    } else {
      v = tile[a][b];
      const int orow = r0 + a, ocol = c0 + b;
      if (orow >= s.out_rows || ocol >= s.out_cols) continue;
      o = s.frag ? frag_off(orow, ocol, s.ldo) : (long long)orow * s.ldo + ocol;
    }
    if (s.e2h) {
      _Float16 h, l;
      split2h_dev(v, exp2i(*s.e2h), h, l);
      reinterpret_cast<_Float16*>(out)[o] = h;
      reinterpret_cast<_Float16*>(out)[o + s.po] = l;
      continue;
    }
    const __bf16 h = (__bf16)v;
    const float r1 = v - (float)h;
    const __bf16 m = (__bf16)r1;
    out[o] = h;
    out[o + s.po] = m;
    out[o + 2 * s.po] = (__bf16)(r1 - (float)m);
  }
}

// fp32 [rows][ld] -> planes out[q][row][col], no LDS (4 columns per thread, 16-B loads when the
// rows allow): a light kernel that co-schedules beside the trunk GEMMs.  out_cols, ldo % 4 == 0.
__global__ __launch_bounds__(256) void split_rows_kernel(SplitParams s, long long per) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int z = blockIdx.y;
  if (gid >= per) return;
  const int c4 = s.out_cols / 4;
  const int r = (int)(gid / c4), c = (int)(gid - (long long)r * c4) * 4;
  const float* x = s.x + z * s.sx + (long long)r * s.ldx;
  float v[4];
  if (r < s.rows && c + 3 < s.cols && (s.ldx & 3) == 0 && (s.sx & 3) == 0 &&
      (reinterpret_cast<unsigned long long>(s.x) & 15) == 0) {
    const float4 a = *reinterpret_cast<const float4*>(x + c);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (r < s.rows && c + j < s.cols) ? x[c + j] : 0.f;
  }
  if (s.e2h) {
    const float sc = exp2i(*s.e2h);
    f16x4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      _Float16 a, b;
      split2h_dev(v[j], sc, a, b);
      h[j] = a; l[j] = b;
    }
    __bf16* o = s.out + z * s.so + (s.frag ? frag_off(r, c, s.ldo) : (long long)r * s.ldo + c);
    *reinterpret_cast<f16x4*>(o) = h;
    *reinterpret_cast<f16x4*>(o + s.po) = l;
    return;
  }
  bf16x4_t h, m, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    __bf16 a, b, cc;
    split3_dev(v[j], a, b, cc);
    h[j] = a; m[j] = b; l[j] = cc;
  }
  __bf16* o = s.out + z * s.so + (s.frag ? frag_off(r, c, s.ldo) : (long long)r * s.ldo + c);
  *reinterpret_cast<bf16x4_t*>(o) = h;
  *reinterpret_cast<bf16x4_t*>(o + s.po) = m;
  *reinterpret_cast<bf16x4_t*>(o + 2 * s.po) = l;
}

// db[z][n] = sum over rows of x[z][rows][n] in two deterministic passes.  Pass 1: a workgroup
// takes 256 columns (4 per lane, 16-B loads) of one row chunk; its 4 waves sum interleaved rows
// (4-deep unrolled) and are added in wave order.  Pass 2: the chunks in order.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x, int rows, int cols, int ld,
                                                             long long sx, int chunks, float* __restrict__ part) {
  __shared__ float4 red[4][64];
  const int z = blockIdx.z, ch = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + 4 * lane;
  const int per = (rows + chunks - 1) / chunks;
  const int r0 = ch * per, r1 = min(rows, r0 + per);
  const float* xp = x + z * sx;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  if (c < cols) {
    int r = r0 + wave;
    for (; r + 4 < r1; r += 8) {
      const float4 a = *reinterpret_cast<const float4*>(xp + (long long)r * ld + c);
      const float4 b = *reinterpret_cast<const float4*>(xp + (long long)(r + 4) * ld + c);
      s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
      s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
    }
    for (; r < r1; r += 4) {
      const float4 a = *reinterpret_cast<const float4*>(xp + (long long)r * ld + c);
      s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
    }
  }
  red[wave][lane] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
  __syncthreads();
  if (wave == 0 && c < cols) {
    const float4 a = red[0][lane], b = red[1][lane], d = red[2][lane], e = red[3][lane];
    const float4 t = make_float4(((a.x + b.x) + d.x) + e.x, ((a.y + b.y) + d.y) + e.y, ((a.z + b.z) + d.z) + e.z,
                                 ((a.w + b.w) + d.w) + e.w);
    *reinterpret_cast<float4*>(part + ((long long)z * chunks + ch) * cols + c) = t;
  }
}

// block: 64 columns x 4 chunk lanes; lane group g sums chunks g, g + 4, ... (8 loads in flight),
// the 4 groups are added in order
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int cols, int chunks,
                                                           float* __restrict__ db, long long sdb) {
  __shared__ float red[4][64];
  const int z = blockIdx.z, cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < cols) {
    const float* pz = part + (long long)z * chunks * cols + c;
    int ch = g;
    for (; ch + 28 < chunks; ch += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pz[(long long)(ch + 4 * u) * cols];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; ch < chunks; ch += 4) s += pz[(long long)ch * cols];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < cols) db[z * sdb + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

// scalar fallback (cols or ld not multiples of 4)
__global__ __launch_bounds__(256) void colsum_partial_scalar_kernel(const float* __restrict__ x, int rows, int cols,
                                                                    int ld, long long sx, int chunks,
                                                                    float* __restrict__ part) {
  const int z = blockIdx.z, c = blockIdx.x * 256 + threadIdx.x, ch = blockIdx.y;
  if (c >= cols) return;
  const int per = (rows + chunks - 1) / chunks;
  const int r0 = ch * per, r1 = min(rows, r0 + per);
  const float* xp = x + z * sx + c;
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += xp[(long long)r * ld];
  part[((long long)z * chunks + ch) * cols + c] = s;
}

}  // namespace

// -1: by operand form; 0: 128x128 k32, 1: 256x128 k32, 2: 256x128 k16, 3: 256x256 k16 (experiments:
// mtsac_debug_x3p_geo, or MTSAC_X3P_GEO at load)
int g_x3p_geo = [] {
  const char* e = getenv("MTSAC_X3P_GEO");
  return e ? atoi(e) : -1;
}();
int g_x3p_dbg = 0;

// tile shape of a geometry id (see Geo aliases above)
static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

static void geo_tile(int geo, int& bm, int& bn) {
  bm = (geo == 0 || geo == 4) ? 128 : geo == 5 ? 224 : 256;
  bn = (geo == 3 || geo == 5) ? 256 : 128;
}

// launch on the instantiation unit of (geometry, operand form)
static void x3p_dispatch(int geo, const SplitGemmParams& p, int epi, int batch, hipStream_t st) {
  int bm, bn;
  geo_tile(geo, bm, bn);
  const unsigned n = (unsigned)(((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn) * batch * (p.splits > 1 ? p.splits : 1));
  const dim3 grid(n);
  if (p.nparts && p.Cp) *p.nparts = (int)n;  // split-K launches write no planes (the finishing pass does)
  const int form = (p.a_kmajor ? 1 : 0) | (p.b_kmajor ? 2 : 0);
  switch (geo) {
    case 0: x3p_unit_g0(p, epi, grid, st); break;
    case 2: x3p_unit_g2(p, epi, grid, st); break;
    case 3:
      if (p.tag == 1) x3p_unit_g3in(p, epi, grid, st);
      else if (form == 0) x3p_unit_g3f0(p, epi, grid, st);
      else if (form == 1) x3p_unit_g3f1(p, epi, grid, st);
      else if (form == 2) x3p_unit_g3f2(p, epi, grid, st);
      else x3p_unit_g3f3(p, epi, grid, st);
      break;
    case 4: x3p_unit_g4(p, epi, grid, st); break;
    case 5:
      if (p.tag == 1 && form == 2) x3p_unit_g5in(p, epi, grid, st);
      else x3p_unit_g5(p, epi, grid, st);
      break;
    default: x3p_unit_g1(p, epi, grid, st); break;
  }
}

// Auto geometry by size (measured, tools/x3p_bench.py): 256x256 tiles (least operand traffic
// per MFMA) when they give >= 192 workgroups or the form is the k-major weight gradient (split-K
// fills the chip there); else 256x128.  g_x3p_geo forces one (experiments).
static int pick_geo(int M, int N, int K, int batch, bool kmajor, bool a_kmajor, int np = 3) {
  if (g_x3p_geo >= 0) return (g_x3p_geo == 5 && a_kmajor) ? 3 : g_x3p_geo;
  // one-plane (bf16) weight grads over few rows (C2: K = 1280): 128 x 128 k32 tiles, two rounds of
  // 256 workgroups for the twin critic and no split-K for the actor -- C2 978-982 -> 991-1007 steps/s
  // against the 256 x 128 k16 tiles (profiles/r5ap_c2_wgrad_geo_ab.txt)
  if (kmajor && np == 1 && K <= 2048) return 0;
  if (kmajor) {  // weight grads over K = rows: 256 x 128 k16 tiles -- measured per launch
                 // (profiles/r3u_wgrad_geo.txt, split3): W = 2048, E = 2, K = 896: 83.9 vs 105.8 us
                 // (no split-K, no reduce pass), K = 1664: 153.8 vs 170.0, K = 3200: 280.3 vs 282.2,
                 // K = 6400: 547.7 vs 541.5 without the 256 x 256 form's slab-reduce pass; W = 400,
                 // E = 2, K = 1280: 26.0 vs 26.6 (128 x 128), K = 6400: 67.0 vs 73.0.  Round 5, whole S3
                 // split2h steps: 5.100 vs 5.128 ms (profiles/r5n_step_ab.txt): the critic's 2 x 128
                 // tiles fill the chip without split-K, so its slabs and reduce pass are gone
    return 2;
  }
  const long long big = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  if (big < 192) return 1;
  if (a_kmajor) return 3;
  // 256- or 224-row tiles: fewer (last-round-padded) rounds x rows per tile
  const long long ncu = cu_count();
  const long long tall = (long long)((M + 223) / 224) * ((N + 255) / 256) * batch;
  return ((tall + ncu - 1) / ncu) * 224 < ((big + ncu - 1) / ncu) * 256 ? 5 : 3;
}

int gemm_x3p_splits(int M, int N, int K, int batch, bool kmajor, int np) {
  int bm, bn;
  geo_tile(pick_geo(M, N, K, batch, kmajor, kmajor, np), bm, bn);
  const long long tiles = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch;
  if (tiles >= 192) return 1;
  // slices: least (rounds of tiles x S workgroups on the CUs) / S, plus a share of a round per
  // extra slice for its partial slab traffic (3 %; 1.5 % for the k-major weight grads, whose
  // 128 x 128 tiles of a W = 400 trunk measured 27 vs 31.5 us at 8 vs 5 slices,
  // profiles/r3f_x3p_w400.txt); >= 8 K-granules per slice (k-major: >= 4)
  const long long ncu = cu_count();
  static const int kdiv = [] {  // experiments: K-granules per slice floor of the k-major form
    const char* e = getenv("MTSAC_X3P_KMAJOR_GRANULES");
    return e && atoi(e) > 0 ? atoi(e) : 4;
  }();
  const int smax = std::min(kmajor ? 16 : 8, std::max(1, K / BK / (kmajor ? kdiv : 8)));
  const double per_slice = kmajor ? 0.015 : 0.03;
  int best = 1;
  double best_cost = 1e30;
  for (int sp = 1; sp <= smax; ++sp) {
    const double cost = (double)((tiles * sp + ncu - 1) / ncu) / sp + per_slice * (sp - 1);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = sp;
    }
  }
  return best;
}

long long gemm_x3p_ws_floats(int M, int N, int K, int batch, bool kmajor) {  // enough for every plane count
  return std::max(gemm_ws_floats(M, N, batch, gemm_x3p_splits(M, N, K, batch, kmajor, 3)),
                  gemm_ws_floats(M, N, batch, gemm_x3p_splits(M, N, K, batch, kmajor, 1)));
}

namespace {

// split-K finish: C = epi(sum_s ws[z*S+s]) (+ its planes), slices added in order
template <int EPI>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(SplitGemmParams p, int S, int batch) {
  const long long slab = (long long)p.M * p.N;
  const int n4 = p.N / 4;
  const long long per = (long long)p.M * n4;
  // split2h planes: the bound's exponent (every block alike) and this block's max |out|
  __shared__ float mscr[16];
  const bool h2 = p.np == 2 && p.Cp;
  float oscale = 1.f, omx = 0.f;
  if (h2) {
    const int ec = gemm_out_exp(p, mscr);
    oscale = exp2i(ec);
    if (blockIdx.x == 0 && threadIdx.x == 0) p.rc->e = ec;
  }
  // grid-stride (a bounded grid: one partial max per block)
  for (long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x; gid < per * batch;
       gid += (long long)gridDim.x * blockDim.x) {
  const int z = (int)(gid / per);
  const long long r = gid - z * per;
  const int row = (int)(r / n4), col = (int)(r - (long long)row * n4) * 4;
  const float* w = p.ws + (long long)z * S * slab + (long long)row * p.N + col;
  float4 v = *reinterpret_cast<const float4*>(w);
  for (int s = 1; s < S; ++s) {
    const float4 u = *reinterpret_cast<const float4*>(w + s * slab);
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  float e[4] = {v.x, v.y, v.z, v.w};
  if (EPI == EPI_BIAS_RELU) {
    const float4 b = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col);
    e[0] = fmaxf(e[0] + b.x, 0.f); e[1] = fmaxf(e[1] + b.y, 0.f);
    e[2] = fmaxf(e[2] + b.z, 0.f); e[3] = fmaxf(e[3] + b.w, 0.f);
  }
  if (EPI == EPI_RELU_MASK && p.mask16 && p.np == 2) {  // fp16 planes: x > 0 <=> h > 0 or l > 0
    const __bf16* mp = p.mask16 + z * p.sMask + (long long)row * p.ldm + col;
    const i16x4 mh = __builtin_bit_cast(i16x4, *reinterpret_cast<const bf16x4_t*>(mp));
    const i16x4 ml = __builtin_bit_cast(i16x4, *reinterpret_cast<const bf16x4_t*>(mp + p.pMask));
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = (mh[j] > 0 || ml[j] > 0) ? e[j] : 0.f;
  } else if (EPI == EPI_RELU_MASK && p.mask16) {  // the activation's bf16 high plane (gemm_x3f nets)
    const bf16x4_t mk = *reinterpret_cast<const bf16x4_t*>(p.mask16 + z * p.sMask + (long long)row * p.ldm + col);
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = (float)mk[j] > 0.f ? e[j] : 0.f;
  } else if (EPI == EPI_RELU_MASK) {
    const float4 mk = *reinterpret_cast<const float4*>(p.mask + z * p.sMask + (long long)row * p.ldm + col);
    e[0] = mk.x > 0.f ? e[0] : 0.f; e[1] = mk.y > 0.f ? e[1] : 0.f;
    e[2] = mk.z > 0.f ? e[2] : 0.f; e[3] = mk.w > 0.f ? e[3] : 0.f;
  }
  if (p.C) *reinterpret_cast<float4*>(p.C + z * p.sC + (long long)row * p.ldc + col) = make_float4(e[0], e[1], e[2], e[3]);
  if (h2) {
    f16x4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      _Float16 a, b;
      split2h_dev(e[j], oscale, a, b);
      h[j] = a; l[j] = b;
      omx = fmaxf(omx, fabsf(e[j]));
    }
    __bf16* cp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
    *reinterpret_cast<f16x4*>(cp) = h;
    *reinterpret_cast<f16x4*>(cp + p.pC) = l;
  } else if (p.Cp) {
    bf16x4_t h, m, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __bf16 a, b, c;
      split3_dev(e[j], a, b, c);
      h[j] = a; m[j] = b; l[j] = c;
    }
    __bf16* cp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
    *reinterpret_cast<bf16x4_t*>(cp) = h;
    if (p.np != 1) {  // precision bf16 reads the high plane only
      *reinterpret_cast<bf16x4_t*>(cp + p.pC) = m;
      *reinterpret_cast<bf16x4_t*>(cp + 2 * p.pC) = l;
    }
  }
  }  // grid-stride
  if (h2) {
    const float m = block_max_val(omx, mscr);
    if (threadIdx.x == 0 && blockIdx.x < PLANE_REC_PARTS) p.rc->amax[blockIdx.x] = m;
  }
}

// the same finish with the bias grad's column-sum partials (p.dbp): block (256 columns, FR rows, z),
// wave w its 4 rows FR chunk + 4 w .. + 3 (loads of all four rows in flight), lane l 4 columns; the
// four waves' column sums meet in LDS and are added in wave order -> dbp[z][row chunk][N]
constexpr int FR = 16;  // rows per finishing block = gemm_x3f's dbp row granularity for split launches
template <int EPI>
__global__ __launch_bounds__(256) void splitk_epilogue_dbp_kernel(SplitGemmParams p, int S) {
  __shared__ float4 red[4][64];
  __shared__ float mscr[16];
  const int z = blockIdx.z, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 256 + 4 * lane;
  const bool cok = col < p.N;
  const long long slab = (long long)p.M * p.N;
  const int nchunks = (p.M + FR - 1) / FR;
  const bool h2 = p.np == 2 && p.Cp;
  float oscale = 1.f, omx = 0.f;
  if (h2) {
    const int ec = gemm_out_exp(p, mscr);
    oscale = exp2i(ec);
    if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) p.rc->e = ec;
  }
  // a bounded grid (one partial max per block): blocks step over the row chunks
  for (int chunk = blockIdx.y; chunk < nchunks; chunk += gridDim.y) {
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 v[4];
  bool ok[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = FR * chunk + 4 * wave + k;
    ok[k] = cok && row < p.M;
    if (ok[k]) v[k] = *reinterpret_cast<const float4*>(p.ws + (long long)z * S * slab + (long long)row * p.N + col);
  }
  for (int s = 1; s < S; ++s) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = FR * chunk + 4 * wave + k;
      if (ok[k]) {
        const float4 u =
            *reinterpret_cast<const float4*>(p.ws + ((long long)z * S + s) * slab + (long long)row * p.N + col);
        v[k].x += u.x; v[k].y += u.y; v[k].z += u.z; v[k].w += u.w;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (!ok[k]) continue;
    const int row = FR * chunk + 4 * wave + k;
    float e[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
    if (EPI == EPI_BIAS_RELU) {
      const float4 b = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col);
      e[0] = fmaxf(e[0] + b.x, 0.f); e[1] = fmaxf(e[1] + b.y, 0.f);
      e[2] = fmaxf(e[2] + b.z, 0.f); e[3] = fmaxf(e[3] + b.w, 0.f);
    }
    if (EPI == EPI_RELU_MASK && p.np == 2) {  // fp16 planes: x > 0 <=> h > 0 or l > 0
      const __bf16* mp = p.mask16 + z * p.sMask + (long long)row * p.ldm + col;
      const i16x4 mh = __builtin_bit_cast(i16x4, *reinterpret_cast<const bf16x4_t*>(mp));
      const i16x4 ml = __builtin_bit_cast(i16x4, *reinterpret_cast<const bf16x4_t*>(mp + p.pMask));
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = (mh[j] > 0 || ml[j] > 0) ? e[j] : 0.f;
    } else if (EPI == EPI_RELU_MASK) {
      const bf16x4_t mk = *reinterpret_cast<const bf16x4_t*>(p.mask16 + z * p.sMask + (long long)row * p.ldm + col);
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = (float)mk[j] > 0.f ? e[j] : 0.f;
    }
    cs.x += e[0]; cs.y += e[1]; cs.z += e[2]; cs.w += e[3];
    if (p.C) *reinterpret_cast<float4*>(p.C + z * p.sC + (long long)row * p.ldc + col) = make_float4(e[0], e[1], e[2], e[3]);
    if (h2) {
      f16x4 h, l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        _Float16 a, b;
        split2h_dev(e[j], oscale, a, b);
        h[j] = a; l[j] = b;
        omx = fmaxf(omx, fabsf(e[j]));
      }
      __bf16* cp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
      *reinterpret_cast<f16x4*>(cp) = h;
      *reinterpret_cast<f16x4*>(cp + p.pC) = l;
    } else if (p.Cp) {
      bf16x4_t h, m, l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __bf16 a, b, c;
        split3_dev(e[j], a, b, c);
        h[j] = a; m[j] = b; l[j] = c;
      }
      __bf16* cp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
      *reinterpret_cast<bf16x4_t*>(cp) = h;
      if (p.np != 1) {
        *reinterpret_cast<bf16x4_t*>(cp + p.pC) = m;
        *reinterpret_cast<bf16x4_t*>(cp + 2 * p.pC) = l;
      }
    }
  }
  red[wave][lane] = cs;
  __syncthreads();
  if (wave == 0 && cok) {
    const float4 a = red[0][lane], b = red[1][lane], c = red[2][lane], d = red[3][lane];
    *reinterpret_cast<float4*>(p.dbp + ((long long)z * nchunks + chunk) * p.N + col) =
        make_float4(((a.x + b.x) + c.x) + d.x, ((a.y + b.y) + c.y) + d.y, ((a.z + b.z) + c.z) + d.z,
                    ((a.w + b.w) + c.w) + d.w);
  }
  __syncthreads();  // red is reused by the next chunk
  cs = make_float4(0.f, 0.f, 0.f, 0.f);
  }  // chunks
  if (h2) {
    const float m = block_max_val(omx, mscr);
    const unsigned b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (threadIdx.x == 0 && b < PLANE_REC_PARTS) p.rc->amax[b] = m;
  }
}

}  // namespace

int splitk_dbp_rows() { return FR; }


void gemm_x3p(const SplitGemmParams& p0, int epi, int batch, hipStream_t st) {
  if (p0.M <= 0 || p0.N <= 0 || p0.K <= 0) return;
  SplitGemmParams p = p0;
  p.dbg |= g_x3p_dbg;
  const bool kmajor = p.a_kmajor && p.b_kmajor;
  const int geo = pick_geo(p.M, p.N, p.K, batch, kmajor, p.a_kmajor != 0, p.np == 0 ? 3 : p.np);
  if (p.splits < 0) p.splits = gemm_x3p_splits(p.M, p.N, p.K, batch, kmajor, p.np == 0 ? 3 : p.np);  // auto
  // split-K: every epilogue works (the finishing pass applies it); the vector finish needs
  // N, ldc, ldm, ldcp multiples of 4
  const bool vec = p.N % 4 == 0 && (!p.C || p.ldc % 4 == 0) && (epi != EPI_RELU_MASK || p.ldm % 4 == 0) &&
                   (!p.Cp || p.ldcp % 4 == 0);
  int S = 1;
  if (p.splits > 1 && p.ws != nullptr && (epi == EPI_STORE && !p.Cp ? true : vec)) {
    const int kt = p.K / BK;
    p.kchunk = (kt + p.splits - 1) / p.splits * BK;
    S = (p.K + p.kchunk - 1) / p.kchunk;
  }
  p.splits = S;
  if (S == 1) p.kchunk = p.K;
  SplitGemmParams q = p;
  int kepi = epi;
  if (S > 1) {  // the GEMM writes raw partial slabs
    q.Cp = nullptr;
    kepi = EPI_STORE;
  }
  // k-major weight grads with arrival counters: the last slice of each tile reduces in-launch
  int bm, bn;
  geo_tile(geo, bm, bn);
  const bool fin = S > 1 && epi == EPI_STORE && !p.Cp && kmajor && p.np != 1 && p.np != 2 && p.cnt != nullptr &&
                   p.N % 4 == 0 && p.ldc % 4 == 0 &&
                   (long long)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn) * batch <= GEMM_X3F_CNT;
  if (!fin) q.cnt = nullptr;
  x3p_dispatch(geo, q, kepi, batch, st);
  const bool cs = p.cs_part != nullptr && p.cs_chunks > 0;
  // defer: the caller runs this finish later, with its network's other ones, in one launch
  const bool defer = epi == EPI_STORE && !p.Cp && p.defer != nullptr && p.defer->n < FINISH_SINK_JOBS;
  if (S == 1 || fin) {
    if (cs && defer) p.defer->job[p.defer->n++] = colsum_job(p.cs_part, p.N, p.cs_chunks, p.cs_db, p.cs_sdb);
    else if (cs) colsum_finish(p.cs_part, p.N, p.cs_chunks, batch, p.cs_db, p.cs_sdb, st);
    return;
  }
  if (epi == EPI_STORE && !p.Cp) {  // the slab sums and (cs) the bias grad's column sums: one launch
    GemmParams r{};
    r.M = p.M;
    r.N = p.N;
    r.C = p.C;
    r.ldc = p.ldc;
    r.sC = p.sC;
    r.ws = p.ws;
    if (defer) p.defer->job[p.defer->n++] = reduce_job(r, batch, S, cs ? p.cs_part : nullptr, p.cs_chunks, p.cs_db, p.cs_sdb);
    else splitk_reduce(r, batch, S, st, cs ? p.cs_part : nullptr, p.cs_chunks, p.cs_db, p.cs_sdb);
    return;
  }
  if (cs) colsum_finish(p.cs_part, p.N, p.cs_chunks, batch, p.cs_db, p.cs_sdb, st);
  splitk_finish(p, epi, S, batch, st);
}

void splitk_finish(const SplitGemmParams& p, int epi, int S, int batch, hipStream_t st) {
  if (p.dbp != nullptr && (epi == EPI_BIAS_RELU || (epi == EPI_RELU_MASK && p.mask16))) {
    // at most PLANE_REC_PARTS blocks (one partial max each, split2h): blocks step over row chunks
    const int gx = (p.N + 255) / 256, chunks = (p.M + FR - 1) / FR;
    const int gy = std::max(1, std::min(chunks, PLANE_REC_PARTS / std::max(1, gx * batch)));
    const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)batch);
    if (p.nparts) *p.nparts = gx * gy * batch;
    if (epi == EPI_BIAS_RELU) hipLaunchKernelGGL(splitk_epilogue_dbp_kernel<EPI_BIAS_RELU>, grid, dim3(256), 0, st, p, S);
    else hipLaunchKernelGGL(splitk_epilogue_dbp_kernel<EPI_RELU_MASK>, grid, dim3(256), 0, st, p, S);
    return;
  }
  const long long n = (long long)batch * p.M * (p.N / 4);
  const dim3 grid((unsigned)std::min<long long>((n + 255) / 256, PLANE_REC_PARTS));
  if (p.nparts) *p.nparts = (int)grid.x;
  if (epi == EPI_BIAS_RELU)
    hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_BIAS_RELU>, grid, dim3(256), 0, st, p, S, batch);
  else if (epi == EPI_RELU_MASK)
    hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_RELU_MASK>, grid, dim3(256), 0, st, p, S, batch);
  else
    hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_STORE>, grid, dim3(256), 0, st, p, S, batch);
}

void split_planes(const SplitParams& s, bool transpose, int batch, hipStream_t st) {
  if (!transpose && s.out_cols % 4 == 0 && s.ldo % 4 == 0 && s.po % 4 == 0 && (batch == 1 || s.so % 4 == 0)) {
    const long long per = (long long)s.out_rows * (s.out_cols / 4);
    hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((per + 255) / 256), batch), dim3(256), 0, st, s, per);
    return;
  }
  dim3 grid((s.rows + 63) / 64, (s.cols + 63) / 64, batch);
  if (transpose)
    hipLaunchKernelGGL(split_kernel<true>, grid, dim3(256), 0, st, s);
  else
    hipLaunchKernelGGL(split_kernel<false>, grid, dim3(256), 0, st, s);
}

void colsum_finish(const float* part, int cols, int chunks, int batch, float* db, long long sdb, hipStream_t st) {
  hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 63) / 64, 1, batch), dim3(256), 0, st, part, cols, chunks, db,
                     sdb);
}

void colsum(const float* x, int rows, int cols, int ld, long long sx, int batch, float* part, float* db,
            long long sdb, hipStream_t st) {
  // ~256 rows per chunk keeps every lane streaming; COLSUM_CHUNKS bounds the partials
  const int chunks = std::max(1, std::min(COLSUM_CHUNKS, (rows + 255) / 256));
  if (cols % 4 == 0 && ld % 4 == 0 && sx % 4 == 0)
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((cols + 255) / 256, chunks, batch), dim3(256), 0, st, x, rows, cols,
                       ld, sx, chunks, part);
  else
    hipLaunchKernelGGL(colsum_partial_scalar_kernel, dim3((cols + 255) / 256, chunks, batch), dim3(256), 0, st, x,
                       rows, cols, ld, sx, chunks, part);
  colsum_finish(part, cols, chunks, batch, db, sdb, st);
}

}  // namespace mtsac
