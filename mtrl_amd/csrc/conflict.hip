// conflict.hip -- eval-time gradient-conflict statistics over per-task gradients (gfx950).
//
// MTSAC.compute_weights (mtrl/rl/algorithms/mtsac.py:870-1170) turns the T per-task gradients of
// a network (flattened in flax ravel order: a T x P matrix G, P = 17.4 M for the MT50/W2048 critic)
// into T x T Gram / cosine / conflict / support / interference matrices
// (compute_gram_metrics :733-771, compute_support_metrics :774-867, vmap_cos_sim and
// compute_conflict_metrics, algorithms/utils.py:49-174).  The reference materialises T x T x P
// boolean tensors; here every O(T^2 P) quantity is one streaming pass over G (HBM-bound reads,
// pair work in registers) and the host finishes the T x T algebra:
//   * task_select: the two order statistics of |g_t| around the support quantile
//     (jnp.quantile 'linear', :804-806) per task -- MSB-first radix select on the float bits
//     (|g| >= 0, so the bit pattern orders like the value), 4 passes of 8 bits, both ranks in
//     the same passes;
//   * task_pair_stats: per column chunk staged in LDS as [column][task], each thread owns a 4 x 4
//     block of task pairs and accumulates g_i . g_j (fp32 per chunk, fp64 across chunks),
//     #(g_i g_j < 0) (the fp32 product, as the reference's sign test), #(S_i & S_j),
//     #(S_i & S_j & g_i g_j < 0) and #(|g_i| < eps & |g_j| > tau) (compute_sparsity_mismatch),
//     plus per-task sum |g| and #(|g| < eps) on the diagonal blocks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "kernels.h"

namespace mtsac {
namespace {

constexpr int TP = 64;           // task rows padded (engine limit: 64 tasks)
constexpr int CH = 64;           // columns per chunk
constexpr int LDT = TP + 4;      // LDS row stride of the [column][task] chunk image
constexpr int NCNT = 4;          // pair counters: conflict, intersection, genuine, mismatch

// ------------------------------------------------------------------ radix select
// One pass: for every task t (blockIdx.y), histogram bits [shift, shift + 8) of |g| over the
// elements whose higher bits equal the current prefix, for both wanted ranks.
__global__ __launch_bounds__(256) void select_hist_kernel(const float* __restrict__ G, long long P,
                                                          const unsigned* __restrict__ prefix /*[T][2]*/,
                                                          unsigned* __restrict__ hist /*[T][2][256]*/, int shift) {
  __shared__ unsigned h[2][256];
  const int t = blockIdx.y;
  for (int i = threadIdx.x; i < 512; i += 256) h[i >> 8][i & 255] = 0;
  __syncthreads();
  const unsigned hi_mask = shift >= 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
  const unsigned p0 = prefix[2 * t] & hi_mask, p1 = prefix[2 * t + 1] & hi_mask;
  const float* g = G + (long long)t * P;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    const unsigned u = __float_as_uint(g[i]) & 0x7FFFFFFFu;  // |g|
    const unsigned d = (u >> shift) & 255u;
    if ((u & hi_mask) == p0) atomicAdd(&h[0][d], 1u);
    if ((u & hi_mask) == p1) atomicAdd(&h[1][d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const unsigned v = h[i >> 8][i & 255];
    if (v) atomicAdd(&hist[(long long)t * 512 + i], v);
  }
}

// per task and rank: the digit whose cumulative count passes the remaining rank; narrows the
// prefix and the rank, clears the histogram for the next pass
__global__ void select_pick_kernel(unsigned* __restrict__ hist, unsigned* __restrict__ prefix,
                                   long long* __restrict__ rank, int T, int shift) {
  const int k = threadIdx.x;  // t * 2 + which
  if (k >= 2 * T) return;
  unsigned* h = hist + (long long)k * 256;
  long long r = rank[k], acc = 0;
  int d = 255;
  for (int i = 0; i < 256; ++i) {
    if (acc + h[i] > r) {
      d = i;
      break;
    }
    acc += h[i];
  }
  rank[k] = r - acc;
  prefix[k] |= (unsigned)d << shift;
  for (int i = 0; i < 256; ++i) h[i] = 0;
}

// ------------------------------------------------------------------ pair statistics
__global__ __launch_bounds__(256) void pair_stats_kernel(const float* __restrict__ G, int T, long long P,
                                                         const float* __restrict__ thr, float eps, float tau,
                                                         double* __restrict__ gram_part /*[grid][TP*TP]*/,
                                                         unsigned long long* __restrict__ counts /*[NCNT][TP*TP]*/,
                                                         double* __restrict__ l1_part /*[grid][TP]*/,
                                                         unsigned long long* __restrict__ nz_count /*[TP]*/) {
  __shared__ __attribute__((aligned(16))) float g[CH][LDT];
  __shared__ float th[TP];
  const int tid = threadIdx.x;
  const int a = tid >> 4, b = tid & 15;  // task rows 4a..4a+3 x 4b..4b+3
  if (tid < TP) th[tid] = tid < T ? thr[tid] : 0.f;
  double gacc[4][4];
  unsigned cnt[NCNT][4][4];
  double l1[4] = {0, 0, 0, 0};
  unsigned nz[4] = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      gacc[r][s] = 0.0;
#pragma unroll
      for (int q = 0; q < NCNT; ++q) cnt[q][r][s] = 0;
    }
  const long long nchunks = (P + CH - 1) / CH;
  for (long long ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const long long c0 = ch * CH;
    __syncthreads();  // the previous chunk's readers are done
    for (int i = tid; i < TP * CH; i += 256) {
      const int t = i / CH, c = i % CH;
      g[c][t] = (t < T && c0 + c < P) ? G[(long long)t * P + c0 + c] : 0.f;
    }
    __syncthreads();
    const int ncol = (int)((P - c0) < CH ? (P - c0) : CH);
    float facc[4][4];
    float fl1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int s = 0; s < 4; ++s) facc[r][s] = 0.f;
    for (int c = 0; c < ncol; ++c) {
      const float4 va = *reinterpret_cast<const float4*>(&g[c][4 * a]);
      const float4 vb = *reinterpret_cast<const float4*>(&g[c][4 * b]);
      const float x[4] = {va.x, va.y, va.z, va.w}, y[4] = {vb.x, vb.y, vb.z, vb.w};
      bool sx[4], sy[4], zx[4], ly[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sx[r] = fabsf(x[r]) >= th[4 * a + r];
        sy[r] = fabsf(y[r]) >= th[4 * b + r];
        zx[r] = fabsf(x[r]) < eps;
        ly[r] = fabsf(y[r]) > tau;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float pr = x[r] * y[s];
          facc[r][s] += pr;
          const bool conf = pr < 0.f;
          const bool joint = sx[r] && sy[s];
          cnt[0][r][s] += conf;
          cnt[1][r][s] += joint;
          cnt[2][r][s] += joint && conf;
          cnt[3][r][s] += zx[r] && ly[s];
        }
      if (a == b) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          fl1[r] += fabsf(x[r]);
          nz[r] += zx[r];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      l1[r] += (double)fl1[r];
#pragma unroll
      for (int s = 0; s < 4; ++s) gacc[r][s] += (double)facc[r][s];
    }
  }
  double* gp = gram_part + (long long)blockIdx.x * TP * TP;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int i = 4 * a + r, j = 4 * b + s;
      gp[i * TP + j] = gacc[r][s];
      if (i < T && j < T) {
#pragma unroll
        for (int q = 0; q < NCNT; ++q)
          if (cnt[q][r][s]) atomicAdd(&counts[(long long)q * TP * TP + i * TP + j], (unsigned long long)cnt[q][r][s]);
      }
    }
  if (a == b) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      l1_part[(long long)blockIdx.x * TP + 4 * a + r] = l1[r];
      if (4 * a + r < T && nz[r]) atomicAdd(&nz_count[4 * a + r], (unsigned long long)nz[r]);
    }
  }
}

// out[k] = sum over parts of part[p][k], fixed order (deterministic)
__global__ void sum_parts_kernel(const double* __restrict__ part, int nparts, int n, double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  double s = 0.0;
  for (int p = 0; p < nparts; ++p) s += part[(long long)p * n + k];
  out[k] = s;
}

__global__ void scatter_blocks_kernel(const float* __restrict__ src, long long src_off, long long src_ms,
                                      float* __restrict__ dst, long long P, long long dst_off, long long dst_ms, int E,
                                      int T, long long blk) {
  const int e = blockIdx.z, t = blockIdx.y;
  const float* s = src + src_off + e * src_ms + t * blk;
  float* d = dst + (long long)t * P + dst_off + e * dst_ms + t * blk;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < blk; i += (long long)gridDim.x * blockDim.x)
    d[i] = s[i];
}

__global__ void check_interleaved_kernel(const int* __restrict__ task, int B, int T_l, int* err) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B && task[r] != r % T_l) atomicOr(err, 1);
}

}  // namespace

void task_select(const float* G, int T, long long P, const long long* ranks /*host [T][2]*/, float* values /*host*/,
                 unsigned* ws_prefix, long long* ws_rank, unsigned* ws_hist, hipStream_t st) {
  (void)hipMemsetAsync(ws_prefix, 0, sizeof(unsigned) * 2 * T, st);
  (void)hipMemsetAsync(ws_hist, 0, sizeof(unsigned) * 512 * T, st);
  (void)hipMemcpyAsync(ws_rank, ranks, sizeof(long long) * 2 * T, hipMemcpyHostToDevice, st);
  const int bx = (int)std::min<long long>((P + 255) / 256, 256);
  for (int shift = 24; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(select_hist_kernel, dim3(bx, T), dim3(256), 0, st, G, P, ws_prefix, ws_hist, shift);
    hipLaunchKernelGGL(select_pick_kernel, dim3(1), dim3(128), 0, st, ws_hist, ws_prefix, ws_rank, T, shift);
  }
  std::vector<unsigned> pre(2 * T);
  (void)hipMemcpyAsync(pre.data(), ws_prefix, sizeof(unsigned) * 2 * T, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  for (int k = 0; k < 2 * T; ++k) {
    float f;
    std::memcpy(&f, &pre[k], sizeof(f));
    values[k] = f;
  }
}

void task_pair_stats(const float* G, int T, long long P, const float* thr /*device [T]*/, float eps, float tau,
                     int grid, double* ws_gram_part /*[grid][64*64]*/, double* ws_l1_part /*[grid][64]*/,
                     unsigned long long* counts /*[4][64*64]*/, unsigned long long* nz /*[64]*/,
                     double* gram /*[64*64]*/, double* l1 /*[64]*/, hipStream_t st) {
  (void)hipMemsetAsync(counts, 0, sizeof(unsigned long long) * NCNT * TP * TP, st);
  (void)hipMemsetAsync(nz, 0, sizeof(unsigned long long) * TP, st);
  (void)hipMemsetAsync(ws_l1_part, 0, sizeof(double) * grid * TP, st);
  hipLaunchKernelGGL(pair_stats_kernel, dim3(grid), dim3(256), 0, st, G, T, P, thr, eps, tau, ws_gram_part, counts,
                     ws_l1_part, nz);
  hipLaunchKernelGGL(sum_parts_kernel, dim3(TP * TP / 256), dim3(256), 0, st, ws_gram_part, grid, TP * TP, gram);
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(TP), 0, st, ws_l1_part, grid, TP, l1);
}

void scatter_task_blocks(const float* src, long long src_off, long long src_ms, float* dst, long long P,
                         long long dst_off, long long dst_ms, int E, int T, long long blk, hipStream_t st) {
  const int bx = (int)std::min<long long>((blk + 255) / 256, 64);
  hipLaunchKernelGGL(scatter_blocks_kernel, dim3(bx, T, E), dim3(256), 0, st, src, src_off, src_ms, dst, P, dst_off,
                     dst_ms, E, T, blk);
}

void check_interleaved(const int* task, int B, int T_l, int* err, hipStream_t st) {
  hipLaunchKernelGGL(check_interleaved_kernel, dim3((B + 255) / 256), dim3(256), 0, st, task, B, T_l, err);
}

}  // namespace mtsac
