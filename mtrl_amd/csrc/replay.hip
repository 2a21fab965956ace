// replay.hip -- device-resident multi-task replay buffer: index stream + gather.
//
// Reference: MultiTaskReplayBuffer (mtrl/rl/buffers.py:221-549).
//
// HBM layout (DESIGN.md "Replay buffer"): one transition RECORD per (slot, task),
//   record = [obs (D) | action (A) | reward | done | next_obs (D) | pad]  (R floats,
//   R = round_up(2D + A + 2, 4)),  store = [capacity][T_local][R].
// A sampled index i therefore selects ONE contiguous slab of T_local * R floats
// (36.8 KB at MT50), which the gather kernel streams with coalesced 4-byte lanes
// straight into the GEMM-ready input matrices (padded, zero-filled widths).
#include "devrng.h"
#include "gemm_common.h"
#include "kernels.h"

namespace mtsac {

// ------------------------------------------------------------------ index stream
// Reproduces Generator.integers(0, high, size=n) (int64, high <= 2**32) of numpy's
// PCG64: random_bounded_uint64_fill -> buffered_bounded_lemire_uint32, whose
// 32-bit words come from pcg64_next32 (low half first, high half buffered).
// A candidate u is accepted iff lo32(u * high) >= (2**32 - high) % high, so the
// draws are "the accepted candidates, in stream order": each lane of ONE wave
// advances the LCG by (lane + 1) steps with a precomputed jump (A_j, C_j) and
// offers two candidates (lo, hi); a ballot prefix count places the accepted ones.
__global__ __launch_bounds__(64) void replay_indices_kernel(PcgDev* rng, const unsigned long long* __restrict__ jump,
                                                            const long long* __restrict__ buf_size, int n,
                                                            int* __restrict__ idx, long long exact_high) {
  const int lane = threadIdx.x;
  const long long size = exact_high > 0 ? exact_high : *buf_size;
  // max(pos or cap, n) (buffers.py:525); exact_high > 0: integers(0, exact_high) as given
  const long long high = exact_high > 0 ? exact_high : (size > n ? size : (long long)n);
  if (high <= 1) {
    for (int i = lane; i < n; i += 64) idx[i] = 0;  // rng == 0: no stream consumption
    return;
  }
  const unsigned int hi32 = (unsigned int)high;  // high < 2**31 (checked at create)
  const unsigned int threshold = (0xFFFFFFFFu - (hi32 - 1u)) % hi32;

  u128 s = {rng->state_hi, rng->state_lo};
  const u128 inc = {rng->inc_hi, rng->inc_lo};
  int has32 = rng->has_uint32;
  const unsigned int buffered = rng->uinteger;
  int produced = 0;

  if (has32) {  // the buffered high half is the first candidate
    has32 = 0;
    const unsigned long long m = (unsigned long long)buffered * hi32;
    if ((unsigned int)m >= threshold) {
      if (lane == 0) idx[0] = (int)(m >> 32);
      produced = 1;
    }
  }
  if (produced >= n) {
    if (lane == 0) rng->has_uint32 = 0;
    return;
  }
  const u128 Aj = {jump[4 * (lane + 1) + 0], jump[4 * (lane + 1) + 1]};
  const u128 Cj = {jump[4 * (lane + 1) + 2], jump[4 * (lane + 1) + 3]};
  const u128 A64 = {jump[4 * 64 + 0], jump[4 * 64 + 1]};
  const u128 C64 = {jump[4 * 64 + 2], jump[4 * 64 + 3]};
  const unsigned long long below = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));

  while (true) {
    const u128 sj = add128(mul128(Aj, s), mul128(Cj, inc));  // state after lane+1 steps
    const unsigned long long o = pcg64_output(sj);
    const unsigned int c_lo = (unsigned int)o, c_hi = (unsigned int)(o >> 32);
    const unsigned long long m_lo = (unsigned long long)c_lo * hi32;
    const unsigned long long m_hi = (unsigned long long)c_hi * hi32;
    const bool a_lo = (unsigned int)m_lo >= threshold;
    const bool a_hi = (unsigned int)m_hi >= threshold;
    const unsigned long long B_lo = __ballot(a_lo);
    const unsigned long long B_hi = __ballot(a_hi);
    const int before = __popcll(B_lo & below) + __popcll(B_hi & below);
    const int pos_lo = produced + before;
    const int pos_hi = pos_lo + (a_lo ? 1 : 0);
    if (a_lo && pos_lo < n) idx[pos_lo] = (int)(m_lo >> 32);
    if (a_hi && pos_hi < n) idx[pos_hi] = (int)(m_hi >> 32);
    const int total = __popcll(B_lo) + __popcll(B_hi);
    if (produced + total >= n) {
      // the candidate that yielded draw n-1 fixes the final generator state
      if (a_lo && pos_lo == n - 1) {
        rng->state_hi = sj.hi;
        rng->state_lo = sj.lo;
        rng->has_uint32 = 1;
        rng->uinteger = c_hi;
      } else if (a_hi && pos_hi == n - 1) {
        rng->state_hi = sj.hi;
        rng->state_lo = sj.lo;
        rng->has_uint32 = 0;
        rng->uinteger = c_hi;  // pcg64_next32 leaves the consumed high word in place
      }
      return;
    }
    produced += total;
    s = add128(mul128(A64, s), mul128(C64, inc));
    (void)has32;
  }
}

void replay_indices(PcgDev* rng, const unsigned long long* jump, const long long* buf_size, int n, int* idx_out,
                    hipStream_t st) {
  hipLaunchKernelGGL(replay_indices_kernel, dim3(1), dim3(64), 0, st, rng, jump, buf_size, n, idx_out, 0LL);
}

void replay_indices_high(PcgDev* rng, const unsigned long long* jump, long long high, int n, int* idx_out,
                         hipStream_t st) {
  hipLaunchKernelGGL(replay_indices_kernel, dim3(1), dim3(64), 0, st, rng, jump, nullptr, n, idx_out, high);
}

// ------------------------------------------------------------------ gather
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ inline int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ inline int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// One wave per output row.  SRC_STORE: rows come from the device buffer through idx
// (row b = i * T_l + t, buffers.py:541-548); otherwise from a user batch.
template <bool SRC_STORE>
__global__ __launch_bounds__(256) void gather_kernel(GatherParams p, const float* __restrict__ u_obs,
                                                     const float* __restrict__ u_act, const float* __restrict__ u_nobs,
                                                     const float* __restrict__ u_done, const float* __restrict__ u_rew,
                                                     int B) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int D = p.obs_dim, A = p.act_dim;
  const int t = b % p.T_l;
  const float* rec = nullptr;
  if (SRC_STORE) {
    const int i = b / p.T_l;
    rec = p.store + ((long long)p.idx[i] * p.T_l + t) * p.R;
  }
  float* xa = p.xa + (long long)b * p.ld_a;
  float* xan = p.xa_next + (long long)b * p.ld_a;
  float* xc = p.xc + (long long)b * p.ld_c;
  float* xcn = p.xc_next + (long long)b * p.ld_c;
  float* xcp = p.xc_pi + (long long)b * p.ld_c;
  const int oh0 = D - p.T_glob;  // first one-hot column
  // split2h: one exponent for every input plane tensor of the step, from the stored rows' max
  const bool h2 = p.in_rec != nullptr;
  const int ein = h2 ? plane_exp(fmaxf(*p.in_max, 1.0f)) : 0;
  const float sin = h2 ? exp2i(ein) : 1.f;
  if (h2 && blockIdx.x == 0 && threadIdx.x == 0) p.in_rec->e = ein;
  // the planes of the same entries: x = h + m + l (split3_dev), or split2h's two fp16 planes
  auto put = [h2, sin](__bf16* q, long long ps, long long o, float x) {
    if (h2) {
      _Float16 h, l;
      split2h_dev(x, sin, h, l);
      reinterpret_cast<_Float16*>(q)[o] = h;
      reinterpret_cast<_Float16*>(q)[o + ps] = l;
      return;
    }
    __bf16 h, m, l;
    split3_dev(x, h, m, l);
    q[o] = h;
    q[o + ps] = m;
    q[o + 2 * ps] = l;
  };
  const long long oa = (long long)b * p.pa_ld, oan = (p.pa_next + b) * p.pa_ld, oc = (long long)b * p.pc_ld;
  int ones = 0, first = 0x7fffffff, bad = 0, n_ones = 0, n_first = 0x7fffffff, n_bad = 0;
  for (int c = lane; c < D; c += 64) {
    const float v = SRC_STORE ? rec[c] : u_obs[(long long)b * D + c];
    const float w = SRC_STORE ? rec[D + A + 2 + c] : u_nobs[(long long)b * D + c];
    xa[c] = v;
    xc[A + c] = v;
    xcp[A + c] = v;
    xan[c] = w;
    xcn[A + c] = w;
    if (p.pa) {
      put(p.pa, p.pa_ps, oa + c, v);
      put(p.pa, p.pa_ps, oan + c, w);
      put(p.pc, p.pc_ps, oc + A + c, v);
      put(p.pcp, p.pc_ps, oc + A + c, v);
      put(p.pcn, p.pc_ps, oc + A + c, w);
    }
    if (c >= oh0) {
      if (v == 1.0f) { ++ones; first = min(first, c - oh0); }
      else if (v != 0.0f) bad = 1;
      if (w == 1.0f) { ++n_ones; n_first = min(n_first, c - oh0); }
      else if (w != 0.0f) n_bad = 1;
    }
  }
  if (lane < A) {
    const float a = SRC_STORE ? rec[D + lane] : u_act[(long long)b * A + lane];
    xc[lane] = a;
    if (p.pa) put(p.pc, p.pc_ps, oc + lane, a);
  }
  ones = wave_sum_i(ones);
  n_ones = wave_sum_i(n_ones);
  bad = wave_sum_i(bad + n_bad);
  first = wave_min_i(first);
  n_first = wave_min_i(n_first);
  if (lane == 0) {
    float r = SRC_STORE ? rec[D + A] : u_rew[b];
    const float d = SRC_STORE ? rec[D + A + 1] : u_done[b];
    if (SRC_STORE && p.rmin != nullptr) {
      const double mn = p.rmin[t], mx = p.rmax[t];
      r = (float)(((double)r - mn) / (mx - mn + p.norm_eps));  // buffers.py:536-538 in float64
    }
    p.rew[b] = r;
    p.done[b] = d;
    int local = first - p.task_begin;
    const bool ok = ones == 1 && n_ones == 1 && bad == 0 && first == n_first && local >= 0 && local < p.T_l;
    if (!ok) {
      atomicOr(p.err, 1);
      local = 0;
    }
    p.task[b] = local;
  }
}

void replay_gather(const GatherParams& p, hipStream_t st) {
  const int B = p.n * p.T_l;
  hipLaunchKernelGGL((gather_kernel<true>), dim3((B + 3) / 4), dim3(256), 0, st, p, nullptr, nullptr, nullptr,
                     nullptr, nullptr, B);
}

void batch_scatter(const GatherParams& p, const float* obs, const float* act, const float* nobs, const float* done,
                   const float* rew, int B, hipStream_t st) {
  hipLaunchKernelGGL((gather_kernel<false>), dim3((B + 3) / 4), dim3(256), 0, st, p, obs, act, nobs, done, rew, B);
}

// ------------------------------------------------------------------ synthetic fill (bench)
// SURVEY.md §8d recipe: obs[:D-T] ~ N(0,1), one-hot of the slot's task, actions U(-1,1),
// rewards U(0,10), dones Bernoulli(1/500); one thread per record.
__device__ inline void atomic_max_abs(float* m, float v) {  // v >= 0: the float order is the bits' order
  atomicMax(reinterpret_cast<unsigned*>(m), __float_as_uint(v));
}

__global__ __launch_bounds__(256) void fill_kernel(float* __restrict__ store, long long nrec, int T_l, int R, int D,
                                                   int A, int T_glob, int task_begin, unsigned long long seed,
                                                   float* bufmax) {
  __shared__ float mscr[16];
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float mx = 0.f;
  if (r < nrec) {
  const int t = (int)(r % T_l);
  float* rec = store + r * R;
  const int F = D - T_glob;
  float nz[4];
  for (int c = 0; c < F; c += 4) {
    normal4(seed, 1u, (unsigned long long)r, (uint32_t)c, nz);
    for (int j = 0; j < 4 && c + j < F; ++j) rec[c + j] = nz[j];
    normal4(seed, 2u, (unsigned long long)r, (uint32_t)c, nz);
    for (int j = 0; j < 4 && c + j < F; ++j) rec[D + A + 2 + c + j] = nz[j];
  }
  for (int c = 0; c < T_glob; ++c) {
    const float v = (c == task_begin + t) ? 1.0f : 0.0f;
    rec[F + c] = v;
    rec[D + A + 2 + F + c] = v;
  }
  float u[4];
  uniform4(seed, 3u, (unsigned long long)r, 0u, u);
  for (int j = 0; j < A && j < 4; ++j) rec[D + j] = 2.0f * u[j] - 1.0f;
  uniform4(seed, 4u, (unsigned long long)r, 0u, u);
  rec[D + A] = 10.0f * u[0];
  rec[D + A + 1] = (u[1] < (1.0f / 500.0f)) ? 1.0f : 0.0f;
  for (int c = 2 * D + A + 2; c < R; ++c) rec[c] = 0.0f;
  for (int c = 0; c < D + A; ++c) mx = fmaxf(mx, fabsf(rec[c]));
  for (int c = D + A + 2; c < 2 * D + A + 2; ++c) mx = fmaxf(mx, fabsf(rec[c]));
  }
  mx = block_max_val(mx, mscr);
  if (threadIdx.x == 0 && bufmax) atomic_max_abs(bufmax, mx);
}

void fill_synthetic(float* store, long long cap, int T_l, int R, int obs_dim, int act_dim, int T_glob, int task_begin,
                    unsigned long long seed, hipStream_t st, float* bufmax) {
  const long long nrec = cap * T_l;
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, st, store, nrec, T_l, R,
                     obs_dim, act_dim, T_glob, task_begin, seed, bufmax);
}

// *m = max(*m, max |x[0..n)|)  (one block; the split2h input bound of a user batch)
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, long long n, float* m) {
  __shared__ float mscr[16];
  float v = 0.f;
  for (long long i = threadIdx.x; i < n; i += 256) v = fmaxf(v, fabsf(x[i]));
  v = block_max_val(v, mscr);
  if (threadIdx.x == 0) *m = fmaxf(*m, v);
}

void absmax_into(const float* x, long long n, float* m, hipStream_t st) {
  hipLaunchKernelGGL(absmax_kernel, dim3(1), dim3(256), 0, st, x, n, m);
}

// ------------------------------------------------------------------ per-task row lists
// Stable counting sort of rows by local task (single workgroup; T_l <= 64).
__global__ __launch_bounds__(256) void task_rows_kernel(const int* __restrict__ task, int B, int T_l,
                                                        int* __restrict__ counts, int* __restrict__ rows,
                                                        int max_rows) {
  __shared__ int cnt[256][65];
  const int tid = threadIdx.x;
  const int chunk = (B + 255) / 256;
  const int r0 = tid * chunk, r1 = min(B, r0 + chunk);
  for (int t = 0; t < T_l; ++t) cnt[tid][t] = 0;
  for (int r = r0; r < r1; ++r) cnt[tid][task[r]] += 1;
  __syncthreads();
  if (tid < T_l) {
    int run = 0;
    for (int j = 0; j < 256; ++j) {
      const int c = cnt[j][tid];
      cnt[j][tid] = run;
      run += c;
    }
    counts[tid] = run;
  }
  __syncthreads();
  for (int r = r0; r < r1; ++r) {
    const int t = task[r];
    const int o = cnt[tid][t]++;
    if (o < max_rows) rows[t * max_rows + o] = r;
  }
}

void task_rows(const int* task, int B, int T_l, int* counts, int* rows, int max_rows, hipStream_t st) {
  hipLaunchKernelGGL(task_rows_kernel, dim3(1), dim3(256), 0, st, task, B, T_l, counts, rows, max_rows);
}

}  // namespace mtsac

namespace mtsac {
namespace {

// One transition slot (T_l records) from five device arrays (T_l rows each) into store[slot]
// (buffers.py:426-474 add: obs[pos] = obs, ...); one thread per record float.
__global__ __launch_bounds__(256) void pack_slot_kernel(float* __restrict__ rec, int T_l, int R, int D, int A,
                                                        const float* __restrict__ obs,
                                                        const float* __restrict__ nobs,
                                                        const float* __restrict__ act,
                                                        const float* __restrict__ rew,
                                                        const float* __restrict__ done) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T_l * R) return;
  const int t = i / R, c = i - t * R;
  float v = 0.f;
  if (c < D) v = obs[t * D + c];
  else if (c < D + A) v = act[t * A + (c - D)];
  else if (c == D + A) v = rew[t];
  else if (c == D + A + 1) v = done[t];
  else if (c < 2 * D + A + 2) v = nobs[t * D + (c - D - A - 2)];
  rec[i] = v;
}

// after the slot is written: running per-task reward min / max in float64 (buffers.py:460-462)
// and the sampled range pos-or-capacity (buffers.py:523) -- device-side, so adds never block
__global__ __launch_bounds__(64) void commit_slot_kernel(const float* __restrict__ rec, int T_l, int R, int rcol,
                                                         double* rmin, double* rmax, long long* buf_size,
                                                         long long size, int D, float* bufmax) {
  const int t = threadIdx.x;
  if (rmin != nullptr && t < T_l) {
    const double r = (double)rec[t * R + rcol];
    rmin[t] = fmin(rmin[t], r);
    rmax[t] = fmax(rmax[t], r);
  }
  if (t == 0) *buf_size = size;
  if (bufmax) {  // the stored rows' max |obs|, |action|, |next_obs| (split2h input planes' bound)
    float m = 0.f;
    for (int i = t; i < T_l * R; i += 64) {
      const int c = i % R;
      if (c < rcol || (c >= rcol + 2 && c < rcol + 2 + D)) m = fmaxf(m, fabsf(rec[i]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (t == 0) atomicMax(reinterpret_cast<unsigned*>(bufmax), __float_as_uint(m));
  }
}

}  // namespace

void buffer_pack_slot(float* rec, int T_l, int R, int D, int A, const float* obs, const float* nobs,
                      const float* act, const float* rew, const float* done, hipStream_t st) {
  const int n = T_l * R;
  hipLaunchKernelGGL(pack_slot_kernel, dim3((n + 255) / 256), dim3(256), 0, st, rec, T_l, R, D, A, obs, nobs, act, rew,
                     done);
}

void buffer_commit_slot(const float* rec, int T_l, int R, int rcol, double* rmin, double* rmax, long long* buf_size,
                        long long size, hipStream_t st, int D, float* bufmax) {
  hipLaunchKernelGGL(commit_slot_kernel, dim3(1), dim3(64), 0, st, rec, T_l, R, rcol, rmin, rmax, buf_size, size, D,
                     bufmax);
}

}  // namespace mtsac
