// heads.hip -- per-task heads, tanh-Gaussian policy, SAC losses, head backward.
//
// Reference: MultiHeadNetwork head selection (mtrl/nn/multi_head.py:50-66),
// ContinuousActionPolicy + TanhMultivariateNormalDiag (mtrl/rl/networks.py:28-45,
// mtrl/nn/distributions.py:6-16), critic / actor losses (mtsac.py:538-566,
// 631-675).  The reference evaluates ALL T heads on every row and then picks the
// row's own head; here only the selected head is computed (same dot product).
// One wavefront per batch row; the head kernels stream the last trunk activation
// (W floats per row) exactly once.
#include "devrng.h"
#include <algorithm>

#include <cstdlib>

#include "gemm_common.h"
#include "kernels.h"

namespace mtsac {

namespace {

constexpr float LOG2F = 0.69314718055994530942f;
constexpr float HALF_LOG_2PI = 0.91893853320467274178f;

__device__ inline float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ inline float softplusf(float z) {  // jax.nn.softplus = logaddexp(z, 0)
  return fmaxf(z, 0.f) + log1pf(expf(-fabsf(z)));
}

// d clip(v, lo, hi) / dv with jax's maximum/minimum tie rule (0.5 at the bounds)
__device__ inline float clip_grad(float v, float lo, float hi) {
  if (v > lo && v < hi) return 1.f;
  if (v == lo || v == hi) return 0.5f;
  return 0.f;
}

// acc[r][o] = sum_w h_r[w] * Wt[w*HD + o] for R rows of one task, reduced over the wave (every lane
// gets the sums).  W % 4 == 0 (and 16-B aligned rows): lane l takes w = 4l + 256i .. +3 with
// 16-B loads of h and of the head kernel (L2-resident: W*HD floats per task), several i in
// flight; otherwise w = l + 64i.  The order is fixed per W, so every kernel that uses this
// gets bitwise the same head outputs.
// WtT (nullable, W % 4 == 0): the same kernel transposed, [HD][W] -- lane l's 4 weights of output o
// are 16 contiguous bytes, so each of the HD loads reads whole lines (from Wt, lanes 4 HD floats
// apart: every load touches 64 lines); the products and their order are unchanged (bitwise equal)
template <int HD, int R>
__device__ inline void rows_dot(const float* const (&h)[R], const float* __restrict__ Wt, int W, float (&acc)[R][HD],
                                const float* __restrict__ WtT = nullptr) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int o = 0; o < HD; ++o) acc[r][o] = 0.f;
  if (WtT != nullptr && (W & 3) == 0) {
#pragma unroll 2
    for (int w = 4 * lane; w < W; w += 256) {
      float4 hv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) hv[r] = *reinterpret_cast<const float4*>(h[r] + w);
      float wv[4 * HD];  // wv[k HD + o] = Wt[w + k][o], as below
#pragma unroll
      for (int o = 0; o < HD; ++o) {
        const float4 v = *reinterpret_cast<const float4*>(WtT + (long long)o * W + w);
        wv[o] = v.x; wv[HD + o] = v.y; wv[2 * HD + o] = v.z; wv[3 * HD + o] = v.w;
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int o = 0; o < HD; ++o) {  // explicit fmas: the same roundings in every R instance
          float a = acc[r][o];
          a = __builtin_fmaf(hv[r].x, wv[o], a);
          a = __builtin_fmaf(hv[r].y, wv[HD + o], a);
          a = __builtin_fmaf(hv[r].z, wv[2 * HD + o], a);
          a = __builtin_fmaf(hv[r].w, wv[3 * HD + o], a);
          acc[r][o] = a;
        }
    }
  } else if ((W & 3) == 0) {
#pragma unroll 2
    for (int w = 4 * lane; w < W; w += 256) {
      float4 hv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) hv[r] = *reinterpret_cast<const float4*>(h[r] + w);
      float wv[4 * HD];  // 4 w x HD outputs, contiguous and 16-B aligned (w % 4 == 0)
#pragma unroll
      for (int i = 0; i < HD; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(Wt + (long long)w * HD + 4 * i);
        wv[4 * i] = v.x; wv[4 * i + 1] = v.y; wv[4 * i + 2] = v.z; wv[4 * i + 3] = v.w;
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int o = 0; o < HD; ++o) {  // explicit fmas: the same roundings in every R instance
          float a = acc[r][o];
          a = __builtin_fmaf(hv[r].x, wv[o], a);
          a = __builtin_fmaf(hv[r].y, wv[HD + o], a);
          a = __builtin_fmaf(hv[r].z, wv[2 * HD + o], a);
          a = __builtin_fmaf(hv[r].w, wv[3 * HD + o], a);
          acc[r][o] = a;
        }
    }
  } else {
    for (int w = lane; w < W; w += 64) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float hv = h[r][w];
#pragma unroll
        for (int o = 0; o < HD; ++o) acc[r][o] = __builtin_fmaf(hv, Wt[(long long)w * HD + o], acc[r][o]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int o = 0; o < HD; ++o) acc[r][o] = wsum(acc[r][o]);
}

template <int HD>
__device__ inline void head_dot(const float* __restrict__ h, const float* __restrict__ Wt, int W, float (&acc)[HD]) {
  const float* const hr[1] = {h};
  float a[1][HD];
  rows_dot<HD, 1>(hr, Wt, W, a);
#pragma unroll
  for (int o = 0; o < HD; ++o) acc[o] = a[0][o];
}

// ------------------------------------------------------------------ actor head + policy
// Given the head outputs acc (mu | log_std) of row b (task t), sample the tanh-Gaussian action and
// its log-probability; lane j < A owns action dimension j.
template <int HD>
__device__ inline void policy_finish(const PolicyParams& p, int b, int t, const float (&acc)[HD], int lane) {
  const HeadParams& hp = p.head;
  const int A = p.A;
  float term = 0.f;
  // the row's loads before the lane test (a load inside it was waited for at the branch's end, one
  // round trip per row): lanes >= A read lane 0's entries and drop them
  const int lj = lane < A ? lane : 0;
  const float bmu = hp.bh[t * HD + lj], bls = hp.bh[t * HD + A + lj];
  const float eps_in = p.eps != nullptr ? p.eps[(long long)b * A + lj] : 0.f;
  if (lane < A) {
    // pick acc[j], acc[A+j] with a static unroll
    float mu = 0.f, ls = 0.f;
#pragma unroll
    for (int o = 0; o < HD; ++o) {
      if (o == lane) mu = acc[o];
      if (o == lane + A) ls = acc[o];
    }
    mu += bmu;
    ls += bls;
    float eps;
    if (p.eps != nullptr) {
      eps = eps_in;
    } else {
      float nz[4];
      normal4(p.seed, p.stream_id + 16u * (uint32_t)(lane >> 2), *p.counter, (uint32_t)b, nz);
      eps = nz[lane & 3];
    }
    const float lsc = fminf(fmaxf(ls, p.ls_min), p.ls_max);
    const float sigma = expf(lsc);
    const float x = mu + sigma * eps;
    const float a = tanhf(x);
    // MVNDiag base log-prob (eps form) minus the Tanh forward log-det (distrax Tanh)
    term = -0.5f * eps * eps - HALF_LOG_2PI - logf(sigma) - 2.0f * (LOG2F - x - softplusf(-2.0f * x));
    p.a_out[(long long)b * p.ld_a_out + lane] = a;
    if (p.a_out2) p.a_out2[(long long)b * p.ld_a_out2 + lane] = a;
    if (p.a_planes && p.ap_rec) {  // split2h: fp16 planes at the input tensor's exponent
      _Float16 h, l;
      split2h_dev(a, exp2i(p.ap_rec->e), h, l);
      const long long o = (long long)b * p.ap_ld + lane;
      reinterpret_cast<_Float16*>(p.a_planes)[o] = h;
      reinterpret_cast<_Float16*>(p.a_planes)[o + p.ap_ps] = l;
    } else if (p.a_planes) {  // the critic input's planes of the action columns (the obs columns: the gather)
      __bf16 h, m, l;
      split3_dev(a, h, m, l);
      const long long o = (long long)b * p.ap_ld + lane;
      p.a_planes[o] = h;
      p.a_planes[o + p.ap_ps] = m;
      p.a_planes[o + 2 * p.ap_ps] = l;
    }
    if (p.cache) {
      float* c = p.cache + (long long)b * 5 * A;
      c[lane] = mu;
      c[A + lane] = ls;
      c[2 * A + lane] = x;
      c[3 * A + lane] = a;
      c[4 * A + lane] = eps;
    }
  }
  term = wsum(term);
  if (lane == 0) p.logpi[b] = term;
}

// one wavefront per row (rollout: rows without task lists)
template <int HD>
__global__ __launch_bounds__(256) void policy_head_kernel(PolicyParams p) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const HeadParams& hp = p.head;
  if (b >= hp.B) return;
  const int t = hp.task[b];
  float acc[HD];
  {
    const float* const hr[1] = {hp.h + (long long)b * hp.W};
    float a[1][HD];
    rows_dot<HD, 1>(hr, hp.Wh + (long long)t * hp.W * HD, hp.W, a,
                    hp.WhT ? hp.WhT + (long long)t * hp.W * HD : nullptr);
#pragma unroll
    for (int o = 0; o < HD; ++o) acc[o] = a[0][o];
  }
  policy_finish<HD>(p, b, t, acc, lane);
}

// Rows grouped by task (task_rows lists): a workgroup takes 4 RW rows of one task, RW per wave, so
// the task's head kernel is fetched (from L2) once per wave for RW rows; no LDS, so it co-resides
// with the trunk GEMMs running on other streams.  RW = 4 when that still gives a workgroup per CU;
// small task shards take fewer rows per wave (more waves in flight; each row's sums are the same).
template <int HD, int RW>
__device__ inline void policy_head_grouped_body(const PolicyParams& p) {
  constexpr int ROWS = 4 * RW;  // rows per workgroup
  const HeadParams& hp = p.head;
  const int t = blockIdx.x;
  const int n = p.counts[t];
  const int j0 = blockIdx.y * ROWS;
  if (j0 >= n) return;  // uniform over the workgroup
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int* rl = p.rows + (long long)t * p.max_rows;
  int row[RW];
  const float* hr[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int jj = j0 + wave * RW + r;
    row[r] = rl[jj < n ? jj : j0];
    hr[r] = hp.h + (long long)row[r] * hp.W;
  }
  float acc[RW][HD];
  rows_dot<HD, RW>(hr, hp.Wh + (long long)t * hp.W * HD, hp.W, acc,
                   hp.WhT ? hp.WhT + (long long)t * hp.W * HD : nullptr);
#pragma unroll
  for (int r = 0; r < RW; ++r)
    if (j0 + wave * RW + r < n) policy_finish<HD>(p, row[r], t, acc[r], lane);
}

template <int HD, int RW>
__global__ __launch_bounds__(256) void policy_head_grouped_kernel(PolicyParams p) {
  policy_head_grouped_body<HD, RW>(p);
}

// the two policy heads of the merged actor forward (s and s' rows) in one launch (blockIdx.z: which)
template <int HD, int RW>
__global__ __launch_bounds__(256) void policy_head_pair_kernel(PolicyPair pp) {
  policy_head_grouped_body<HD, RW>(pp.p[blockIdx.z]);
}

// rows per wave for a launch that would have wgs_at_rw1 workgroups at one row per wave: the largest
// of 4, 2, 1 that still gives >= 1024 workgroups (four per CU: the row loads of more waves in flight;
// S3, serialised: the policy-head pair 68.7 -> 39.8 us at 2 rows per wave instead of 4, the action
// grad 43.5 -> 30.4 us at 1, profiles/r4t_*)
static int rows_per_wave(long long wgs_at_rw1) {
  static const int forced = [] {  // MTSAC_HEAD_RW=1 / 2 / 4: experiments
    const char* e = getenv("MTSAC_HEAD_RW");
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 2 || v == 4 ? v : 0;
  }();
  if (forced) return forced;
  for (int rw = 4; rw > 1; rw >>= 1)
    if (wgs_at_rw1 / rw >= 1024) return rw;
  return 1;
}

// ------------------------------------------------------------------ critic heads + losses
// grid-stride over rows (one wave per row at a time); split2h: each workgroup's max |dq| to dq_rec
__global__ __launch_bounds__(256) void critic_head_kernel(CriticHeadParams p) {
  const int lane = threadIdx.x & 63;
  const HeadParams& hp = p.head;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  float dqmax = 0.f;
  for (int b = wid; b < hp.B; b += gridDim.x * 4) {
  const int t = hp.task[b];
  float q[4];
  const int E = hp.E;
  for (int e = 0; e < E; ++e) {
    float acc[1];
    head_dot<1>(hp.h + e * hp.sh + (long long)b * hp.W, hp.Wh + e * hp.sWh + (long long)t * hp.W, hp.W, acc);
    q[e] = acc[0] + hp.bh[e * hp.sbh + t];
  }
  float qt[4];  // fused_target: the target critic's heads of the same row (same row, same task)
  if (p.fused_target) {
    const HeadParams& th = p.thead;
    for (int e = 0; e < E; ++e) {
      float acc[1];
      head_dot<1>(th.h + e * th.sh + (long long)b * th.W, th.Wh + e * th.sWh + (long long)t * th.W, th.W, acc);
      qt[e] = acc[0] + th.bh[e * th.sbh + t];
    }
  }
  if (lane != 0) continue;
  const float alpha = expf(p.log_alpha[p.task_begin + t]);  // exp(onehot . log_alpha), mtsac.py:60-63
  float w = 1.f;
  if (p.tw != nullptr) w = p.tw[b];  // T * softmax(-log_alpha)[t] (mtsac.py:103-113)
  auto td_target = [&](const float* qq) {
    float mn = qq[0];
    for (int e = 1; e < E; ++e) mn = fminf(mn, qq[e]);
    const float mnext = mn - alpha * p.logpi[b];
    float y = p.rew[b] + (1.0f - p.done[b]) * p.gamma * mnext;  // mtsac.py:547-553
    if (p.clip) y = fminf(fmaxf(y, -5000.f), 5000.f);
    p.y_out[b] = y;
    return y;
  };
  if (p.mode == CH_TARGET) {
    td_target(q);
  } else if (p.mode == CH_CRITIC) {
    const float y = p.fused_target ? td_target(qt) : p.y[b];
    float sq = 0.f, qs = 0.f;
    for (int e = 0; e < E; ++e) {
      float qc = q[e], dcl = 1.f;
      if (p.clip) {
        dcl = clip_grad(qc, -5000.f, 5000.f);
        qc = fminf(fmaxf(qc, -5000.f), 5000.f);
      }
      const float diff = qc - y;
      sq += w * diff * diff;
      qs += qc;
      const float g = w * 2.0f * diff * p.inv_norm * dcl;
      p.dq[e * hp.B + b] = g;
      dqmax = fmaxf(dqmax, fabsf(g));
    }
    p.row_a[b] = sq;
    p.row_b[b] = qs;
  } else {  // CH_ACTOR: loss = mean(w * (alpha*logpi - min_k Q_k))   mtsac.py:659-666
    float mn = q[0];
    for (int e = 1; e < E; ++e) mn = fminf(mn, q[e]);
    int cnt = 0;
    for (int e = 0; e < E; ++e) cnt += (q[e] == mn) ? 1 : 0;
    for (int e = 0; e < E; ++e) {
      const float g = (q[e] == mn) ? (-w * p.inv_norm / (float)cnt) : 0.f;
      p.dq[e * hp.B + b] = g;
      dqmax = fmaxf(dqmax, fabsf(g));
    }
    p.row_a[b] = w * (alpha * p.logpi[b] - mn);
    p.alpha_w[b] = w * alpha * p.inv_norm;
  }
  }  // rows
  if (p.dq_rec) {  // one max per workgroup (lane 0 of each wave holds its wave's)
    __shared__ float smx[4];
    if (lane == 0) smx[threadIdx.x >> 6] = dqmax;
    __syncthreads();
    if (threadIdx.x == 0) p.dq_rec->amax[blockIdx.x] = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  }
}

// ------------------------------------------------------------------ head backward (data)
// Grouped by task: block (256 columns, task t, row slice rs, member e); the lane's 4 x HD head
// weights stay in registers while wave rl walks the task's rows j = 4 rs + rl + 4 HB_RS k (rows
// from task_rows; two per iteration for loads in flight).  dbp: the (task, slice) column sums
// (the bias gradient's partials, [e][T_l * HB_RS][W]; waves added in order), so the trunk's bias
// grad needs no pass over an fp32 dz.  dz (fp32) may be null.
constexpr int HB_RS = 4;

// the masked data grad of row b at columns w .. w + 3 (loads only)
template <int HD>
__device__ inline float4 head_bwd_val(const HeadParams& hp, const float* __restrict__ dout, long long s_dout, int e,
                                      int b, int w, const float (&wt)[4][HD]) {
  const float* d = dout + e * s_dout + (long long)b * HD;
  float g[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < HD; ++o) s += d[o] * wt[k][o];
    g[k] = s;
  }
  const float4 h = *reinterpret_cast<const float4*>(hp.h + e * hp.sh + (long long)b * hp.W + w);
  float4 out;
  out.x = h.x > 0.f ? g[0] : 0.f;
  out.y = h.y > 0.f ? g[1] : 0.f;
  out.z = h.z > 0.f ? g[2] : 0.f;
  out.w = h.w > 0.f ? g[3] : 0.f;
  return out;
}

// its stores: fp32 dz (if any) and the GEMM planes
template <int HD>
__device__ inline void head_bwd_put(const HeadParams& hp, int e, int b, int w, float4 out, float* __restrict__ dz,
                                    const PlaneOut& po) {
  const long long off = e * hp.sh + (long long)b * hp.W + w;
  if (dz) *reinterpret_cast<float4*>(dz + off) = out;
  if (po.p && po.rc) {  // split2h: fp16 planes at the bound's exponent (oscale folded into po.kmul below)
    const float v[4] = {out.x, out.y, out.z, out.w};
    f16x4 ph, pl;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      _Float16 a, b2;
      split2h_dev(v[k], po.w_add, a, b2);  // w_add carries the block's output scale here (head_bwd_data_body)
      ph[k] = a;
      pl[k] = b2;
    }
    __bf16* q = po.p + e * po.sm + (long long)b * po.ld + w;
    *reinterpret_cast<f16x4*>(q) = ph;
    *reinterpret_cast<f16x4*>(q + po.ps) = pl;
  } else if (po.p) {  // the bf16 split planes the next GEMMs read
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const float v[4] = {out.x, out.y, out.z, out.w};
    bf16x4 ph, pm, pl;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const __bf16 hh = (__bf16)v[k];
      const float r1 = v[k] - (float)hh;
      const __bf16 mm = (__bf16)r1;
      ph[k] = hh;
      pm[k] = mm;
      pl[k] = (__bf16)(r1 - (float)mm);
    }
    __bf16* q = po.p + e * po.sm + (long long)b * po.ld + w;
    *reinterpret_cast<bf16x4*>(q) = ph;
    *reinterpret_cast<bf16x4*>(q + po.ps) = pm;
    *reinterpret_cast<bf16x4*>(q + 2 * po.ps) = pl;
  }
}

template <int HD>
__device__ inline float4 head_bwd_row(const HeadParams& hp, const float* __restrict__ dout, long long s_dout, int e,
                                      int b, int w, const float (&wt)[4][HD], float* __restrict__ dz,
                                      const PlaneOut& po) {
  const float4 out = head_bwd_val<HD>(hp, dout, s_dout, e, b, w, wt);
  head_bwd_put<HD>(hp, e, b, w, out, dz, po);
  return out;
}

// ------------------------------------------------------------------ checked LDS reductions
// Every cross-wave LDS reduction of the head backward is checked: the wave that reads the other
// waves' slots keeps a digest of the bits it read, hands it back through `chk`, and after a barrier
// each writer compares it with the digest of the registers it stored.  A slot that did not hold its
// writer's bits when it was read ORs a HEAD_FAULT_* bit into HeadParams::fault; the engine turns that
// into an error at the next sync (engine.cpp check_err), so a recurrence of the round-5 event (one
// wrong head weight-grad value on an emulated rank whose inputs were right) fails
// loudly instead of as a tolerance miss.  The digests cost a few VALU ops and one barrier per block.
__device__ inline unsigned digest4(unsigned d, float4 v) {
  d = __builtin_rotateleft32(d, 5) ^ __float_as_uint(v.x);
  d = __builtin_rotateleft32(d, 5) ^ __float_as_uint(v.y);
  d = __builtin_rotateleft32(d, 5) ^ __float_as_uint(v.z);
  return __builtin_rotateleft32(d, 5) ^ __float_as_uint(v.w);
}
__device__ inline void head_fault(unsigned* fault, unsigned bit) {
  if (fault) __hip_atomic_fetch_or(fault, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (bx, by, bz) of a [W / 256][T_l HB_RS][E] grid; red: 4 x 64 float4 of LDS, chk: 4 x 64 digests
template <int HD>
__device__ inline void head_bwd_data_body(const HeadParams& hp, const float* __restrict__ dout, long long s_dout,
                                          float* __restrict__ dz, const PlaneOut& po_in, float* __restrict__ dbp,
                                          const int* __restrict__ counts, const int* __restrict__ rows, int max_rows,
                                          int bx, int by, int bz, int gy, float4 (*red)[64], unsigned (*chk)[64]) {
  // split2h: the planes' exponent from the bound kmul * max|dout| * (max|head weight| + w_add), every
  // workgroup alike (red is the scratch of the maxima); the scale rides in po.w_add from here on
  PlaneOut po = po_in;
  if (po.p && po.rc) {
    const float md = rec_max(po.rd, po.nd, reinterpret_cast<float*>(red));
    const int ec = plane_exp(po.kmul * md * (po.rw->amax[1] + po.w_add));
    po.w_add = exp2i(ec);
    if (bx == 0 && by == 0 && bz == 0 && threadIdx.x == 0) po.rc->e = ec;
  }
  const int e = bz, t = by / HB_RS, rs = by - t * HB_RS;
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int w = bx * 256 + 4 * lane;
  const bool ok = w < hp.W;
  const int n = counts[t];
  const int* rw = rows + (long long)t * max_rows;
  float wt[4][HD];
  if (ok) {
    const float* Wt = hp.Wh + e * hp.sWh + ((long long)t * hp.W + w) * HD;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int o = 0; o < HD; ++o) wt[k][o] = Wt[k * HD + o];
  }
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok && n > 0) {
    // CH rows per batch: their row indices, then their loads, all unconditional (clamped to the last
    // row) so they are in flight together; the stores and sums of the rows past n are dropped.  Rows
    // are added in ascending j as before.
    constexpr int STRIDE = 4 * HB_RS, CH = 4;
    for (int j0 = 4 * rs + rl; j0 < n; j0 += CH * STRIDE) {
      int bb[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) bb[u] = rw[min(j0 + u * STRIDE, n - 1)];
      float4 o[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) o[u] = head_bwd_val<HD>(hp, dout, s_dout, e, bb[u], w, wt);
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (j0 + u * STRIDE >= n) break;
        head_bwd_put<HD>(hp, e, bb[u], w, o[u], dz, po);
        cs.x += o[u].x; cs.y += o[u].y; cs.z += o[u].z; cs.w += o[u].w;
      }
    }
  }
  if (dbp == nullptr) return;
  red[rl][lane] = cs;
  const unsigned own = digest4(0u, cs);
  __syncthreads();
  if (rl == 0 && ok) {
    const float4 a = red[0][lane], b = red[1][lane], c = red[2][lane], d = red[3][lane];
    *reinterpret_cast<float4*>(dbp + ((long long)e * gy + by) * hp.W + w) =
        make_float4(((a.x + b.x) + c.x) + d.x, ((a.y + b.y) + c.y) + d.y, ((a.z + b.z) + c.z) + d.z,
                    ((a.w + b.w) + c.w) + d.w);
    chk[0][lane] = digest4(0u, a);
    chk[1][lane] = digest4(0u, b);
    chk[2][lane] = digest4(0u, c);
    chk[3][lane] = digest4(0u, d);
  }
  __syncthreads();
  if (ok && chk[rl][lane] != own) head_fault(hp.fault, HEAD_FAULT_COLSUM);
}

template <int HD>
__global__ __launch_bounds__(256) void head_bwd_data_kernel(HeadParams hp, const float* __restrict__ dout,
                                                            long long s_dout, float* __restrict__ dz, PlaneOut po,
                                                            float* __restrict__ dbp, const int* __restrict__ counts,
                                                            const int* __restrict__ rows, int max_rows) {
  __shared__ float4 red[4][64];
  __shared__ unsigned chk[4][64];
  head_bwd_data_body<HD>(hp, dout, s_dout, dz, po, dbp, counts, rows, max_rows, blockIdx.x, blockIdx.y, blockIdx.z,
                         gridDim.y, red, chk);
}

// ------------------------------------------------------------------ head backward (weights)
// dWh[t][w][o] = sum over the task's rows of h[row][w] dout[row][o]; wave g sums rows j = g mod 4
// in order, then the four waves are added in order (same association in both kernels).
template <int HD>
__global__ __launch_bounds__(256) void head_bwd_weight_scalar_kernel(HeadParams hp, const float* __restrict__ dout,
                                                              long long s_dout, const int* __restrict__ counts,
                                                              const int* __restrict__ rows, int max_rows,
                                                              float* __restrict__ dWh, float* __restrict__ dbh) {
  __shared__ float red[4][64][HD];
  const int t = blockIdx.x;
  const int w0 = blockIdx.y * 64;
  const int e = blockIdx.z;
  const int wl = threadIdx.x & 63;
  const int rg = threadIdx.x >> 6;
  const int w = w0 + wl;
  const int n = counts[t];
  const int* rl = rows + (long long)t * max_rows;
  const float* h = hp.h + e * hp.sh;
  const float* d = dout + e * s_dout;
  float acc[HD];
#pragma unroll
  for (int o = 0; o < HD; ++o) acc[o] = 0.f;
  if (w < hp.W) {
#pragma unroll 8
    for (int j = rg; j < n; j += 4) {
      const int row = rl[j];
      const float hv = h[(long long)row * hp.W + w];
#pragma unroll
      for (int o = 0; o < HD; ++o) acc[o] += hv * d[(long long)row * HD + o];
    }
  }
#pragma unroll
  for (int o = 0; o < HD; ++o) red[rg][wl][o] = acc[o];
  __syncthreads();
  if (rg == 0 && w < hp.W) {
    float* out = dWh + e * hp.sWh + ((long long)t * hp.W + w) * HD;
#pragma unroll
    for (int o = 0; o < HD; ++o) out[o] = red[0][wl][o] + red[1][wl][o] + red[2][wl][o] + red[3][wl][o];
  }
  if (blockIdx.y == 0) {  // bias grad: 256 strided partial sums, then a fixed-order tree
    __syncthreads();
    float* part = &red[0][0][0];  // 256 * HD floats
#pragma unroll
    for (int o = 0; o < HD; ++o) {
      float s = 0.f;
      for (int j = threadIdx.x; j < n; j += 256) s += d[(long long)rl[j] * HD + o];
      part[o * 256 + threadIdx.x] = s;
    }
    __syncthreads();
    for (int half = 128; half > 0; half >>= 1) {
      if (threadIdx.x < half)
#pragma unroll
        for (int o = 0; o < HD; ++o) part[o * 256 + threadIdx.x] += part[o * 256 + threadIdx.x + half];
      __syncthreads();
    }
    if (threadIdx.x < HD) dbh[e * hp.sbh + t * HD + threadIdx.x] = part[threadIdx.x * 256];
  }
}

// W % 4 == 0: each lane owns 4 consecutive w (16-B loads), a workgroup 256 w; (bx, by, bz) of a
// [T_l][W / 256][E] grid; red: HD x 4 x 64 float4 of LDS ([o][wave][lane]: a wave's 64 lanes write one
// contiguous KiB, no bank conflicts), chk: 4 x 64 digests
template <int HD, bool INJECT = false>
__device__ inline void head_bwd_weight_body(const HeadParams& hp, const float* __restrict__ dout, long long s_dout,
                                            const int* __restrict__ counts, const int* __restrict__ rows, int max_rows,
                                            float* __restrict__ dWh, float* __restrict__ dbh, int bx, int by, int bz,
                                            float4 (*red)[4][64], unsigned (*chk)[64]) {
  const int t = bx, e = bz;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = by * 256 + 4 * lane;
  const int n = counts[t];
  const int* rl = rows + (long long)t * max_rows;
  const float* h = hp.h + e * hp.sh;
  const float* d = dout + e * s_dout;
  float4 acc[HD];
#pragma unroll
  for (int o = 0; o < HD; ++o) acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (w < hp.W) {
#pragma unroll 8
    for (int j = wave; j < n; j += 4) {
      const int row = rl[j];
      const float4 hv = *reinterpret_cast<const float4*>(h + (long long)row * hp.W + w);
#pragma unroll
      for (int o = 0; o < HD; ++o) {
        const float dv = d[(long long)row * HD + o];
        acc[o].x += hv.x * dv;
        acc[o].y += hv.y * dv;
        acc[o].z += hv.z * dv;
        acc[o].w += hv.w * dv;
      }
    }
  }
  unsigned own = 0u;
#pragma unroll
  for (int o = 0; o < HD; ++o) {
    red[o][wave][lane] = acc[o];
    own = digest4(own, acc[o]);
  }
  if constexpr (INJECT) {  // the self-check's own test (mtsac_debug_head_selfcheck): one slot gets other bits
    if (wave == 1 && lane == 48) red[HD - 1][1][48].x = __uint_as_float(__float_as_uint(acc[HD - 1].x) ^ 1u);
  }
  __syncthreads();
  if (wave == 0 && w < hp.W) {
    float v[4][HD];
    unsigned dg[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int o = 0; o < HD; ++o) {
      const float4 a0 = red[o][0][lane], a1 = red[o][1][lane], a2 = red[o][2][lane], a3 = red[o][3][lane];
      v[0][o] = a0.x + a1.x + a2.x + a3.x;
      v[1][o] = a0.y + a1.y + a2.y + a3.y;
      v[2][o] = a0.z + a1.z + a2.z + a3.z;
      v[3][o] = a0.w + a1.w + a2.w + a3.w;
      dg[0] = digest4(dg[0], a0);
      dg[1] = digest4(dg[1], a1);
      dg[2] = digest4(dg[2], a2);
      dg[3] = digest4(dg[3], a3);
    }
    float* out = dWh + e * hp.sWh + ((long long)t * hp.W + w) * HD;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int o = 0; o < HD; ++o) out[k * HD + o] = v[k][o];
#pragma unroll
    for (int g = 0; g < 4; ++g) chk[g][lane] = dg[g];
  }
  __syncthreads();  // also orders wave 0's reads of red before the bias pass reuses it
  if (w < hp.W && chk[wave][lane] != own) head_fault(hp.fault, HEAD_FAULT_WGRAD);
  if (by == 0) {  // bias grad: 256 strided partial sums, then a fixed-order tree
    float* part = reinterpret_cast<float*>(&red[0][0][0]);  // >= 256 * HD floats
#pragma unroll
    for (int o = 0; o < HD; ++o) {
      float s = 0.f;
      for (int j = threadIdx.x; j < n; j += 256) s += d[(long long)rl[j] * HD + o];
      part[o * 256 + threadIdx.x] = s;
    }
    __syncthreads();
    for (int half = 128; half > 0; half >>= 1) {
      if (threadIdx.x < half)
#pragma unroll
        for (int o = 0; o < HD; ++o) part[o * 256 + threadIdx.x] += part[o * 256 + threadIdx.x + half];
      __syncthreads();
    }
    if (threadIdx.x < HD) dbh[e * hp.sbh + t * HD + threadIdx.x] = part[threadIdx.x * 256];
  }
}

template <int HD>
__global__ __launch_bounds__(256) void head_bwd_weight_kernel(HeadParams hp, const float* __restrict__ dout,
                                                              long long s_dout, const int* __restrict__ counts,
                                                              const int* __restrict__ rows, int max_rows,
                                                              float* __restrict__ dWh, float* __restrict__ dbh) {
  __shared__ float4 red[HD][4][64];
  __shared__ unsigned chk[4][64];
  head_bwd_weight_body<HD>(hp, dout, s_dout, counts, rows, max_rows, dWh, dbh, blockIdx.x, blockIdx.y, blockIdx.z,
                           red, chk);
}

// head_bwd_weight_kernel with one LDS slot corrupted on purpose (the self-check's test, never in a step)
template <int HD>
__global__ __launch_bounds__(256) void head_bwd_weight_inject_kernel(HeadParams hp, const float* __restrict__ dout,
                                                                     long long s_dout, const int* __restrict__ counts,
                                                                     const int* __restrict__ rows, int max_rows,
                                                                     float* __restrict__ dWh, float* __restrict__ dbh) {
  __shared__ float4 red[HD][4][64];
  __shared__ unsigned chk[4][64];
  head_bwd_weight_body<HD, true>(hp, dout, s_dout, counts, rows, max_rows, dWh, dbh, blockIdx.x, blockIdx.y,
                                 blockIdx.z, red, chk);
}

// Both halves of a head's backward in ONE launch (they read the same dout and are independent):
// blocks [0, nd) are head_bwd_data's [W / 256][T_l HB_RS][E] grid, the rest head_bwd_weight's
// [T_l][W / 256][E] grid -- the same arithmetic per block, one launch fewer per network.
template <int HD>
__global__ __launch_bounds__(256) void head_bwd_both_kernel(HeadParams hp, const float* __restrict__ dout,
                                                            long long s_dout, float* __restrict__ dz, PlaneOut po,
                                                            float* __restrict__ dbp, const int* __restrict__ counts,
                                                            const int* __restrict__ rows, int max_rows, int T_l,
                                                            float* __restrict__ dWh, float* __restrict__ dbh) {
  __shared__ float4 red[HD][4][64];
  __shared__ unsigned chk[4][64];
  const int gw = (hp.W + 255) / 256, gy = T_l * HB_RS;
  const int nd = gw * gy * hp.E;
  int b = blockIdx.x;
  if (b < nd) {
    const int bx = b % gw, by = (b / gw) % gy, bz = b / (gw * gy);
    head_bwd_data_body<HD>(hp, dout, s_dout, dz, po, dbp, counts, rows, max_rows, bx, by, bz, gy,
                           reinterpret_cast<float4 (*)[64]>(&red[0][0][0]), chk);
    return;
  }
  b -= nd;
  const int bx = b % T_l, by = (b / T_l) % gw, bz = b / (T_l * gw);
  head_bwd_weight_body<HD>(hp, dout, s_dout, counts, rows, max_rows, dWh, dbh, bx, by, bz, red, chk);
}

// The head backward's data and weight passes reading h ONCE: block (task t, 256 columns bx, member e),
// wave g walks the task's rows j = g, g + 4, ... (the weight pass's order) in batches of four, row
// u of a batch being row slice rs = u of the data pass (j = 4 rs + g + 16 k): per row the masked data
// grad (planes out), its column sum into the (t, rs) partial, and h dout into the weight grad.  Every
// output is bitwise the separate passes' (head_bwd_data_body / head_bwd_weight_body): the same
// products, added in the same order.
template <int HD>
__global__ __launch_bounds__(256) void head_bwd_fused_kernel(HeadParams hp, const float* __restrict__ dout,
                                                             long long s_dout, float* __restrict__ dz, PlaneOut po,
                                                             float* __restrict__ dbp, const int* __restrict__ counts,
                                                             const int* __restrict__ rows, int max_rows, int T_l,
                                                             float* __restrict__ dWh, float* __restrict__ dbh) {
  constexpr int HDL = HD < HB_RS ? HB_RS : HD;  // the column-sum reduction needs [HB_RS][4][64] float4
  __shared__ float4 red[HDL][4][64];               // weight sums: [o][wave][lane]
  __shared__ unsigned chk[4][64], rchk[HB_RS][4][64];  // the reductions' digests (checked LDS reductions)
  const int gw = (hp.W + 255) / 256, gy = T_l * HB_RS;
  const int t = blockIdx.x % T_l, bx = (blockIdx.x / T_l) % gw, e = blockIdx.x / (T_l * gw);
  if (po.p && po.rc) {  // split2h: as head_bwd_data_body
    const float md = rec_max(po.rd, po.nd, reinterpret_cast<float*>(&red[0][0][0]));
    const int ec = plane_exp(po.kmul * md * (po.rw->amax[1] + po.w_add));
    po.w_add = exp2i(ec);
    if (blockIdx.x == 0 && threadIdx.x == 0) po.rc->e = ec;
    __syncthreads();  // the scratch is red: reused below
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = bx * 256 + 4 * lane;
  const bool ok = w < hp.W;
  const int n = counts[t];
  const int* rl = rows + (long long)t * max_rows;
  const float* h = hp.h + e * hp.sh;
  const float* d = dout + e * s_dout;
  float wt[4][HD];
  if (ok) {
    const float* Wt = hp.Wh + e * hp.sWh + ((long long)t * hp.W + w) * HD;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int o = 0; o < HD; ++o) wt[k][o] = Wt[k * HD + o];
  }
  float4 acc[HD], cs[HB_RS];
#pragma unroll
  for (int o = 0; o < HD; ++o) acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < HB_RS; ++u) cs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok && n > 0) {
    for (int j0 = wave; j0 < n; j0 += 4 * HB_RS) {
      int bb[HB_RS];
#pragma unroll
      for (int u = 0; u < HB_RS; ++u) bb[u] = rl[min(j0 + 4 * u, n - 1)];
      float4 hv[HB_RS];
      float dv[HB_RS][HD];
#pragma unroll
      for (int u = 0; u < HB_RS; ++u) {
        hv[u] = *reinterpret_cast<const float4*>(h + (long long)bb[u] * hp.W + w);
#pragma unroll
        for (int o = 0; o < HD; ++o) dv[u][o] = d[(long long)bb[u] * HD + o];
      }
#pragma unroll
      for (int u = 0; u < HB_RS; ++u) {
        if (j0 + 4 * u >= n) break;
        float g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float s = 0.f;
#pragma unroll
          for (int o = 0; o < HD; ++o) s += dv[u][o] * wt[k][o];
          g[k] = s;
        }
        float4 out;
        out.x = hv[u].x > 0.f ? g[0] : 0.f;
        out.y = hv[u].y > 0.f ? g[1] : 0.f;
        out.z = hv[u].z > 0.f ? g[2] : 0.f;
        out.w = hv[u].w > 0.f ? g[3] : 0.f;
        head_bwd_put<HD>(hp, e, bb[u], w, out, dz, po);
        cs[u].x += out.x; cs[u].y += out.y; cs[u].z += out.z; cs[u].w += out.w;
#pragma unroll
        for (int o = 0; o < HD; ++o) {
          const float dvo = dv[u][o];
          acc[o].x += hv[u].x * dvo;
          acc[o].y += hv[u].y * dvo;
          acc[o].z += hv[u].z * dvo;
          acc[o].w += hv[u].w * dvo;
        }
      }
    }
  }
  // weight grad: the four waves in order (head_bwd_weight_body), checked
  unsigned own = 0u;
#pragma unroll
  for (int o = 0; o < HD; ++o) {
    red[o][wave][lane] = acc[o];
    own = digest4(own, acc[o]);
  }
  __syncthreads();
  if (wave == 0 && ok) {
    float v[4][HD];
    unsigned dg[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int o = 0; o < HD; ++o) {
      const float4 a0 = red[o][0][lane], a1 = red[o][1][lane], a2 = red[o][2][lane], a3 = red[o][3][lane];
      v[0][o] = a0.x + a1.x + a2.x + a3.x;
      v[1][o] = a0.y + a1.y + a2.y + a3.y;
      v[2][o] = a0.z + a1.z + a2.z + a3.z;
      v[3][o] = a0.w + a1.w + a2.w + a3.w;
      dg[0] = digest4(dg[0], a0);
      dg[1] = digest4(dg[1], a1);
      dg[2] = digest4(dg[2], a2);
      dg[3] = digest4(dg[3], a3);
    }
    float* out = dWh + e * hp.sWh + ((long long)t * hp.W + w) * HD;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int o = 0; o < HD; ++o) out[k * HD + o] = v[k][o];
#pragma unroll
    for (int g = 0; g < 4; ++g) chk[g][lane] = dg[g];
  }
  __syncthreads();
  if (ok && chk[wave][lane] != own) head_fault(hp.fault, HEAD_FAULT_WGRAD);
  // the data grad's column sums per row slice rs: waves (a + b) + c + d (head_bwd_data_body), checked
  if (dbp != nullptr) {
    float4(*cr)[4][64] = reinterpret_cast<float4(*)[4][64]>(&red[0][0][0]);  // [rs][wave][lane]
    unsigned owns[HB_RS];
#pragma unroll
    for (int u = 0; u < HB_RS; ++u) {
      cr[u][wave][lane] = cs[u];
      owns[u] = digest4(0u, cs[u]);
    }
    __syncthreads();
    if (ok) {  // wave g finishes row slice rs = g
      const float4 a = cr[wave][0][lane], b = cr[wave][1][lane], c = cr[wave][2][lane], dd = cr[wave][3][lane];
      *reinterpret_cast<float4*>(dbp + ((long long)e * gy + t * HB_RS + wave) * hp.W + w) =
          make_float4(((a.x + b.x) + c.x) + dd.x, ((a.y + b.y) + c.y) + dd.y, ((a.z + b.z) + c.z) + dd.z,
                      ((a.w + b.w) + c.w) + dd.w);
      rchk[wave][0][lane] = digest4(0u, a);
      rchk[wave][1][lane] = digest4(0u, b);
      rchk[wave][2][lane] = digest4(0u, c);
      rchk[wave][3][lane] = digest4(0u, dd);
    }
    __syncthreads();
    if (ok) {
      bool bad = false;
#pragma unroll
      for (int u = 0; u < HB_RS; ++u) bad |= rchk[u][wave][lane] != owns[u];
      if (bad) head_fault(hp.fault, HEAD_FAULT_COLSUM);
    }
  }
  if (bx == 0) {  // head bias grad: as head_bwd_weight_body
    float* part = reinterpret_cast<float*>(&red[0][0][0]);  // >= 256 * HD floats
#pragma unroll
    for (int o = 0; o < HD; ++o) {
      float s = 0.f;
      for (int j = threadIdx.x; j < n; j += 256) s += d[(long long)rl[j] * HD + o];
      part[o * 256 + threadIdx.x] = s;
    }
    __syncthreads();
    for (int half = 128; half > 0; half >>= 1) {
      if (threadIdx.x < half)
#pragma unroll
        for (int o = 0; o < HD; ++o) part[o * 256 + threadIdx.x] += part[o * 256 + threadIdx.x + half];
      __syncthreads();
    }
    if (threadIdx.x < HD) dbh[e * hp.sbh + t * HD + threadIdx.x] = part[threadIdx.x * 256];
  }
}

// ------------------------------------------------------------------ critic -> action grad -> policy grad
// AG_RW rows per wavefront: the critic layer-0 kernel rows (A x Wc) are read once per AG_RW rows
// (4, or fewer on small task shards, see rows_per_wave).  Per row the sums run over the lane's w
// (16-B chunks 4l + 256i when Wc % 4 == 0, else l + 64i), then over the wave.
// AM: action dimensions held per row -- 4 (MetaWorld: no run-time test around the weight loads, which
// were otherwise waited for one at a time) or 8 (any A <= 8)
// rows b0 .. b0 + AG_RW - 1 of one wave; returns the wave's max |dout| (lanes < A; 0 elsewhere)
template <int AG_RW, int AM>
__device__ inline float action_grad_rows(const ActionGradParams& p, int b0, int lane) {
  const int A = p.A;
  int rows[AG_RW];
#pragma unroll
  for (int r = 0; r < AG_RW; ++r) rows[r] = min(b0 + r, p.B - 1);
  float ga[AG_RW][AM];
#pragma unroll
  for (int r = 0; r < AG_RW; ++r)
#pragma unroll
    for (int j = 0; j < AM; ++j) ga[r][j] = 0.f;
  for (int e = 0; e < p.E; ++e) {
    const float* dz = p.dz1 + e * p.s_dz;
    const float* W0 = p.W0 + e * p.s_W0;
    if ((p.Wc & 3) == 0) {  // 16-B loads: lane l takes w = 4l + 256i .. +3
#pragma unroll 2
      for (int w = 4 * lane; w < p.Wc; w += 256) {
        float4 wv[AM];
#pragma unroll
        for (int j = 0; j < AM; ++j)
          wv[j] = (AM == 4 || j < A) ? *reinterpret_cast<const float4*>(W0 + (long long)j * p.Wc + w)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < AG_RW; ++r) {
          const float4 g = *reinterpret_cast<const float4*>(dz + (long long)rows[r] * p.Wc + w);
#pragma unroll
          for (int j = 0; j < AM; ++j) {  // explicit fmas: the same roundings in every AG_RW instance
            float a = ga[r][j];
            a = __builtin_fmaf(g.x, wv[j].x, a);
            a = __builtin_fmaf(g.y, wv[j].y, a);
            a = __builtin_fmaf(g.z, wv[j].z, a);
            a = __builtin_fmaf(g.w, wv[j].w, a);
            ga[r][j] = a;
          }
        }
      }
      continue;
    }
    for (int w = lane; w < p.Wc; w += 64) {
      float wv[AM];
#pragma unroll
      for (int j = 0; j < AM; ++j) wv[j] = (AM == 4 || j < A) ? W0[(long long)j * p.Wc + w] : 0.f;
#pragma unroll
      for (int r = 0; r < AG_RW; ++r) {
        const float g = dz[(long long)rows[r] * p.Wc + w];
#pragma unroll
        for (int j = 0; j < AM; ++j) ga[r][j] = __builtin_fmaf(g, wv[j], ga[r][j]);
      }
    }
  }
  float omx = 0.f;
  // every row's cache entries and temperature weight first (loads outside the row / lane tests)
  const int lj = lane < A ? lane : 0;
  float c_ls[AG_RW], c_a[AG_RW], c_eps[AG_RW], c_lp[AG_RW];
#pragma unroll
  for (int r = 0; r < AG_RW; ++r) {
    const float* c = p.cache + (long long)rows[r] * 5 * A;
    c_ls[r] = c[A + lj];
    c_a[r] = c[3 * A + lj];
    c_eps[r] = c[4 * A + lj];
    c_lp[r] = p.alpha_w[rows[r]];
  }
  // no contraction in the per-row tail: the vectoriser packs rows of the 2- and 4-row instances, and
  // contracted multiply-adds then round differently per instance (profiles/r4v_head_forms.txt)
#pragma unroll
  for (int r = 0; r < AG_RW; ++r) {
#pragma clang fp contract(off)
    const int b = b0 + r;
#pragma unroll
    for (int j = 0; j < AM; ++j) ga[r][j] = j < A ? wsum(ga[r][j]) : 0.f;
    if (b >= p.B || lane >= A) continue;
    float g_a = 0.f;
#pragma unroll
    for (int j = 0; j < AM; ++j)
      if (j == lane) g_a = ga[r][j];
    const float ls = c_ls[r], a = c_a[r], eps = c_eps[r];
    const float g_logpi = c_lp[r];
    const float sigma = expf(fminf(fmaxf(ls, p.ls_min), p.ls_max));
    const float g_x = g_a * (1.0f - a * a) + g_logpi * 2.0f * a;  // d logpi/dx = 2 tanh(x)
    const float g_ls = (g_x * sigma * eps - g_logpi) * clip_grad(ls, p.ls_min, p.ls_max);
    p.dout[(long long)b * 2 * A + lane] = g_x;
    p.dout[(long long)b * 2 * A + A + lane] = g_ls;
    omx = fmaxf(omx, fmaxf(fabsf(g_x), fabsf(g_ls)));
  }
  return omx;
}

// grid-stride over wave row groups (the grid is capped at PLANE_REC_PARTS workgroups); split2h: one
// max |dout| per workgroup (the actor head backward's bound input), every row covered
template <int AG_RW, int AM>
__global__ __launch_bounds__(256) void action_grad_kernel(ActionGradParams p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float omx = 0.f;
  for (int wid = blockIdx.x * 4 + wave; wid * AG_RW < p.B; wid += gridDim.x * 4)
    omx = fmaxf(omx, action_grad_rows<AG_RW, AM>(p, wid * AG_RW, lane));
  if (p.dout_rec) {
    __shared__ float smx[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) omx = fmaxf(omx, __shfl_xor(omx, o));
    if (lane == 0) smx[wave] = omx;
    __syncthreads();
    if (threadIdx.x == 0) p.dout_rec->amax[blockIdx.x] = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  }
}

// ------------------------------------------------------------------ per-row alpha / task weights
__global__ __launch_bounds__(256) void row_alpha_kernel(const int* __restrict__ task, int task_begin,
                                                        const float* __restrict__ log_alpha, int T_glob, int B,
                                                        int use_tw, float* __restrict__ alpha_row,
                                                        float* __restrict__ tw_row) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int tg = task_begin + task[b];
  alpha_row[b] = expf(log_alpha[tg]);
  if (use_tw) {  // T * softmax(-log_alpha)[t]  (mtsac.py:103-113)
    float mx = -log_alpha[0];
    for (int i = 1; i < T_glob; ++i) mx = fmaxf(mx, -log_alpha[i]);
    float s = 0.f;
    for (int i = 0; i < T_glob; ++i) s += expf(-log_alpha[i] - mx);
    tw_row[b] = (expf(-log_alpha[tg] - mx) / s) * (float)T_glob;
  }
}

// WhT[t][o][w] = Wh[t][w][o]: one thread per output element (reads hd-strided, writes whole lines)
__global__ __launch_bounds__(256) void head_transpose_kernel(const float* __restrict__ Wh, int W, int hd,
                                                             long long n, float* __restrict__ WhT) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long per = (long long)W * hd;
  const long long t = i / per, r = i - t * per;
  const int o = (int)(r / W), w = (int)(r - (long long)o * W);
  WhT[i] = Wh[t * per + (long long)w * hd + o];
}

}  // namespace

void head_transpose(const float* Wh, int T_l, int W, int hd, float* WhT, hipStream_t st) {
  const long long n = (long long)T_l * W * hd;
  if (n <= 0) return;
  hipLaunchKernelGGL(head_transpose_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, Wh, W, hd, n, WhT);
}

void policy_head(const PolicyParams& p, hipStream_t st) {
  const int hd = p.head.hd;
  if (p.counts != nullptr) {
    const int rw = rows_per_wave((long long)p.T_l * ((p.max_count + 3) / 4));
    dim3 grid((unsigned)p.T_l, (unsigned)((p.max_count + 4 * rw - 1) / (4 * rw)));
#define PHG(HDV)                                                                                          \
  if (rw == 4) hipLaunchKernelGGL((policy_head_grouped_kernel<HDV, 4>), grid, dim3(256), 0, st, p);        \
  else if (rw == 2) hipLaunchKernelGGL((policy_head_grouped_kernel<HDV, 2>), grid, dim3(256), 0, st, p);   \
  else hipLaunchKernelGGL((policy_head_grouped_kernel<HDV, 1>), grid, dim3(256), 0, st, p);
    if (hd == 8) { PHG(8) }
    else if (hd == 6) { PHG(6) }
    else if (hd == 4) { PHG(4) }
    else { PHG(2) }
#undef PHG
    return;
  }
  dim3 grid((p.head.B + 3) / 4);
  if (hd == 8)
    hipLaunchKernelGGL(policy_head_kernel<8>, grid, dim3(256), 0, st, p);
  else if (hd == 6)
    hipLaunchKernelGGL(policy_head_kernel<6>, grid, dim3(256), 0, st, p);
  else if (hd == 4)
    hipLaunchKernelGGL(policy_head_kernel<4>, grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(policy_head_kernel<2>, grid, dim3(256), 0, st, p);
}

void policy_head_pair(const PolicyParams& a, const PolicyParams& b, hipStream_t st) {
  if (!a.counts || !b.counts || a.head.hd != b.head.hd || a.T_l != b.T_l || a.max_count != b.max_count) {
    policy_head(a, st);
    policy_head(b, st);
    return;
  }
  const int rw = rows_per_wave(2LL * a.T_l * ((a.max_count + 3) / 4));
  const dim3 grid((unsigned)a.T_l, (unsigned)((a.max_count + 4 * rw - 1) / (4 * rw)), 2);
  PolicyPair pp{};
  pp.p[0] = a;
  pp.p[1] = b;
#define PHP(HDV)                                                                                       \
  if (rw == 4) hipLaunchKernelGGL((policy_head_pair_kernel<HDV, 4>), grid, dim3(256), 0, st, pp);       \
  else if (rw == 2) hipLaunchKernelGGL((policy_head_pair_kernel<HDV, 2>), grid, dim3(256), 0, st, pp);  \
  else hipLaunchKernelGGL((policy_head_pair_kernel<HDV, 1>), grid, dim3(256), 0, st, pp);
  if (a.head.hd == 8) { PHP(8) }
  else if (a.head.hd == 6) { PHP(6) }
  else if (a.head.hd == 4) { PHP(4) }
  else { PHP(2) }
#undef PHP
}

void critic_head(const CriticHeadParams& p, hipStream_t st) {
  // a wave per row (grid-stride past PLANE_REC_PARTS workgroups: one max per workgroup, split2h);
  // at S3 6400 rows in flight instead of 2048 waves stepping over three rows each
  const int g = std::min((p.head.B + 3) / 4, PLANE_REC_PARTS);
  if (p.dq_parts) *p.dq_parts = g;
  hipLaunchKernelGGL(critic_head_kernel, dim3(g), dim3(256), 0, st, p);
}

void head_backward_data(const HeadParams& hp, const float* dout, long long s_dout, float* dz, const int* counts,
                        const int* rows, int max_rows, int T_l, hipStream_t st, PlaneOut po, float* dbp) {
  const dim3 grid((unsigned)((hp.W + 255) / 256), (unsigned)(T_l * HB_RS), (unsigned)hp.E);
#define HBD_LAUNCH(HDV)                                                                                  \
  hipLaunchKernelGGL(head_bwd_data_kernel<HDV>, grid, dim3(256), 0, st, hp, dout, s_dout, dz, po, dbp, counts, \
                     rows, max_rows)
  switch (hp.hd) {
    case 1: HBD_LAUNCH(1); break;
    case 2: HBD_LAUNCH(2); break;
    case 4: HBD_LAUNCH(4); break;
    case 6: HBD_LAUNCH(6); break;
    default: HBD_LAUNCH(8); break;
  }
#undef HBD_LAUNCH
}

int head_backward_chunks(int T_l) { return T_l * HB_RS; }

bool head_backward_both(const HeadParams& hp, const float* dout, long long s_dout, float* dz, const int* counts,
                        const int* rows, int max_rows, int T_l, PlaneOut po, float* dbp, float* dWh, float* dbh,
                        hipStream_t st) {
  if (hp.W % 4 != 0) return false;  // the scalar weight kernel: two launches
  const int gw = (hp.W + 255) / 256;
  static const bool split_req = [] {  // MTSAC_HEAD_BWD_SPLIT=1: the data and weight passes as separate blocks
    const char* e = getenv("MTSAC_HEAD_BWD_SPLIT");
    return e && atoi(e) != 0;
  }();
  // the one-pass form has a workgroup per (task, 256 columns, member): below one per CU (task shards,
  // MT10) the separate passes' 5x more workgroups win (7-task shard: 27 / 18 us one-pass against
  // 15 / 11 us, profiles/r4u_sums_t7_split2h.txt vs r4g); bitwise the same either way
  const bool split = split_req || (long long)T_l * gw * hp.E < 256;
  const dim3 grid((unsigned)(split ? gw * T_l * HB_RS * hp.E + T_l * gw * hp.E : T_l * gw * hp.E));
#define HBB_LAUNCH(HDV)                                                                                         \
  if (split)                                                                                                    \
    hipLaunchKernelGGL(head_bwd_both_kernel<HDV>, grid, dim3(256), 0, st, hp, dout, s_dout, dz, po, dbp, counts,  \
                       rows, max_rows, T_l, dWh, dbh);                                                          \
  else                                                                                                          \
    hipLaunchKernelGGL(head_bwd_fused_kernel<HDV>, grid, dim3(256), 0, st, hp, dout, s_dout, dz, po, dbp, counts, \
                       rows, max_rows, T_l, dWh, dbh)
  switch (hp.hd) {
    case 1: HBB_LAUNCH(1); break;
    case 2: HBB_LAUNCH(2); break;
    case 4: HBB_LAUNCH(4); break;
    case 6: HBB_LAUNCH(6); break;
    default: HBB_LAUNCH(8); break;
  }
#undef HBB_LAUNCH
  return true;
}

void head_backward_weight(const HeadParams& hp, const float* dout, long long s_dout, const int* counts,
                          const int* rows, int max_rows, float* dWh, float* dbh, hipStream_t st) {
  const unsigned T_l = (unsigned)(hp.sbh / hp.hd);  // bias stride per member = T_l * hd
#define HBW_LAUNCH(K, HDV, WPB)                                                                             \
  hipLaunchKernelGGL(K<HDV>, dim3(T_l, (hp.W + WPB - 1) / WPB, hp.E), dim3(256), 0, st, hp, dout, s_dout, counts, \
                     rows, max_rows, dWh, dbh)
  const bool vec = hp.W % 4 == 0;
  switch (hp.hd) {
    case 1: if (vec) HBW_LAUNCH(head_bwd_weight_kernel, 1, 256); else HBW_LAUNCH(head_bwd_weight_scalar_kernel, 1, 64); break;
    case 2: if (vec) HBW_LAUNCH(head_bwd_weight_kernel, 2, 256); else HBW_LAUNCH(head_bwd_weight_scalar_kernel, 2, 64); break;
    case 4: if (vec) HBW_LAUNCH(head_bwd_weight_kernel, 4, 256); else HBW_LAUNCH(head_bwd_weight_scalar_kernel, 4, 64); break;
    case 6: if (vec) HBW_LAUNCH(head_bwd_weight_kernel, 6, 256); else HBW_LAUNCH(head_bwd_weight_scalar_kernel, 6, 64); break;
    default: if (vec) HBW_LAUNCH(head_bwd_weight_kernel, 8, 256); else HBW_LAUNCH(head_bwd_weight_scalar_kernel, 8, 64); break;
  }
#undef HBW_LAUNCH
}

void head_backward_weight_inject(const HeadParams& hp, const float* dout, long long s_dout, const int* counts,
                                 const int* rows, int max_rows, int T_l, float* dWh, float* dbh, hipStream_t st) {
  if (hp.hd != 8 || hp.W % 4 != 0) return;  // the instance the round-5 event hit (actor head, hd = 8)
  hipLaunchKernelGGL(head_bwd_weight_inject_kernel<8>, dim3((unsigned)T_l, (unsigned)((hp.W + 255) / 256), (unsigned)hp.E),
                     dim3(256), 0, st, hp, dout, s_dout, counts, rows, max_rows, dWh, dbh);
}

void action_grad(const ActionGradParams& p, hipStream_t st) {
  const int rw = rows_per_wave((p.B + 3) / 4);
  const dim3 grid((unsigned)std::min((p.B + 4 * rw - 1) / (4 * rw), PLANE_REC_PARTS));
  if (p.dout_parts) *p.dout_parts = (int)grid.x;  // one partial max per workgroup
#define AGL(AMV)                                                                                  \
  if (rw == 4) hipLaunchKernelGGL((action_grad_kernel<4, AMV>), grid, dim3(256), 0, st, p);        \
  else if (rw == 2) hipLaunchKernelGGL((action_grad_kernel<2, AMV>), grid, dim3(256), 0, st, p);   \
  else hipLaunchKernelGGL((action_grad_kernel<1, AMV>), grid, dim3(256), 0, st, p);
  if (p.A == 4) { AGL(4) }
  else { AGL(8) }
#undef AGL
}

void row_alpha(const int* task, int task_begin, const float* log_alpha, int T_glob, int B, int use_task_weights,
               float* alpha_row, float* tw_row, hipStream_t st) {
  hipLaunchKernelGGL(row_alpha_kernel, dim3((B + 255) / 256), dim3(256), 0, st, task, task_begin, log_alpha, T_glob,
                     B, use_task_weights, alpha_row, tw_row);
}

}  // namespace mtsac
