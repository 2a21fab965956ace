// gemm_f32.hip -- exact-fp32 MFMA GEMM for the MTSAC trunk layers (gfx950).
//
// Replaces the XLA dots of flax nn.Dense (mtrl/nn/multi_head.py:34-44) and their
// autodiff transposes (jax.value_and_grad at mtrl/rl/algorithms/mtsac.py:587-596,
// 689-691).  Numerics: v_mfma_f32_32x32x2_f32 is a k-ordered f32 fmaf chain, so the
// result is an fp32 dot product with fp32 accumulation (no xf32 / bf16 shortcut).
//
// Tile: 128x128 per 256-thread workgroup, BK = 32, 4 waves in a 2x2 grid, each wave
// 64x64 = 2x2 accumulators of 32x32 (64 AGPR/VGPR).  Global -> registers -> LDS
// staging with the next K-tile's loads in flight during the MFMAs; operands are
// stored k-major in LDS ([k][m], [k][n]) so each MFMA operand is one conflict-free
// ds_read_b32 per lane (lanes 0-31 consecutive m/n, lanes 32-63 the next k row).
#include "gemm_common.h"

namespace mtsac {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 32;
constexpr int NTH = 256;

// Loader shapes (per thread, 4 float4 per operand per K-tile):
//  "transposing": operand stored [rows][K] (reduction contiguous).  f = t + 256 i ->
//                 kq = t & 7 (float4 along k), r = (t >> 3) + 32 i.   LDS [4kq+j][r].
//  "direct":      operand stored [K][cols] (output index contiguous). f = t + 256 i ->
//                 cq = t & 31 (float4 along cols), k = (t >> 5) + 8 i. LDS [k][4cq..].
template <bool TRANSPOSING>
struct Loader {
  static constexpr int PAD = TRANSPOSING ? 1 : 4;  // PAD=1: conflict-free scalar stores; 4: b128
  static constexpr int LD = 128 + PAD;

  __device__ static inline void load(const float* __restrict__ base, int ld, int r0, int nrows, int k0, int K,
                                     float4 (&v)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (TRANSPOSING) {
        const int kq = t & 7;
        const int r = (t >> 3) + 32 * i;
        const int row = r0 + r, k = k0 + 4 * kq;
        if (row < nrows && k < K) x = *reinterpret_cast<const float4*>(base + (long long)row * ld + k);
      } else {
        const int cq = t & 31;
        const int kk = (t >> 5) + 8 * i;
        const int k = k0 + kk, col = r0 + 4 * cq;
        if (k < K && col < nrows) x = *reinterpret_cast<const float4*>(base + (long long)k * ld + col);
      }
      v[i] = x;
    }
  }

  __device__ static inline void store(float* __restrict__ lds, const float4 (&v)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (TRANSPOSING) {
        const int kq = t & 7;
        const int r = (t >> 3) + 32 * i;
        lds[(4 * kq + 0) * LD + r] = v[i].x;
        lds[(4 * kq + 1) * LD + r] = v[i].y;
        lds[(4 * kq + 2) * LD + r] = v[i].z;
        lds[(4 * kq + 3) * LD + r] = v[i].w;
      } else {
        const int cq = t & 31;
        const int kk = (t >> 5) + 8 * i;
        *reinterpret_cast<float4*>(lds + kk * LD + 4 * cq) = v[i];
      }
    }
  }
};

template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(NTH, 2) void gemm_f32_kernel(GemmParams p) {
  // A: TA ? [K][M] (direct) : [M][K] (transposing);  B: TB ? [N][K] (transposing) : [K][N] (direct)
  using LA = Loader<!TA>;
  using LB = Loader<TB>;
  __shared__ float As[BK * LA::LD];
  __shared__ float Bs[BK * LB::LD];

  const GemmSlice sl = gemm_slice<TA, TB>(p);
  const int z = sl.z;
  const float* __restrict__ A = sl.A;
  const float* __restrict__ B = sl.B;
  float* __restrict__ C = sl.C;
  const int K = sl.K;

  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int t = threadIdx.x;
  const int wave = t >> 6;
  const int lane = t & 63;
  const int wm = (wave & 1) * 64;
  const int wn = (wave >> 1) * 64;
  const int lr = lane & 31;
  const int lk = lane >> 5;

  // fused bias-gradient (column sums of B) for weight-grad GEMMs: m-tile 0 only
  const bool do_db = (EPI == EPI_STORE) && !TB && sl.db != nullptr && blockIdx.x == 0;
  float dbacc = 0.f;

  f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};

  float4 ra[4], rb[4];
  const int nk = (K + BK - 1) / BK;
  LA::load(A, p.lda, m0, p.M, 0, K, ra);
  LB::load(B, p.ldb, n0, p.N, 0, K, rb);
  LA::store(As, ra);
  LB::store(Bs, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = (kt + 1) < nk;
    if (more) {
      LA::load(A, p.lda, m0, p.M, (kt + 1) * BK, K, ra);
      LB::load(B, p.ldb, n0, p.N, (kt + 1) * BK, K, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float* ar = As + (kk + lk) * LA::LD + wm + lr;
      const float* br = Bs + (kk + lk) * LB::LD + wn + lr;
      const float a0 = ar[0], a1 = ar[32];
      const float b0 = br[0], b1 = br[32];
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc11, 0, 0, 0);
    }
    if (do_db) {
      const int col = t & 127, half = t >> 7;
#pragma unroll
      for (int r = 0; r < BK / 2; ++r) dbacc += Bs[(half * (BK / 2) + r) * LB::LD + col];
    }
    __syncthreads();
    if (more) {
      LA::store(As, ra);
      LB::store(Bs, rb);
      __syncthreads();
    }
  }

  if (do_db) {
    // combine the two row halves through LDS (As is free now)
    const int col = t & 127, half = t >> 7;
    if (half == 1) As[col] = dbacc;
    __syncthreads();
    if (half == 0 && n0 + col < p.N) sl.db[n0 + col] = dbacc + As[col];
  }

  // epilogue: acc[i][j] element r -> row = (r&3) + 8(r>>2) + 4*lk, col = lr (32x32 C/D map)
  const float* __restrict__ bias = (EPI == EPI_BIAS_RELU) ? p.bias + z * p.sBias : nullptr;
  const float* __restrict__ mask = (EPI == EPI_RELU_MASK) ? p.mask + z * p.sMask : nullptr;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn + 32 * j + lr;
    const bool colok = col < p.N;
    const float bv = (EPI == EPI_BIAS_RELU && colok) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x16 acc = (i == 0) ? (j == 0 ? acc00 : acc01) : (j == 0 ? acc10 : acc11);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < p.M && colok) {
          float v = acc[r];
          if (EPI == EPI_BIAS_RELU) v = fmaxf(v + bv, 0.f);
          if (EPI == EPI_RELU_MASK) v = (mask[(long long)row * p.ldm + col] > 0.f) ? v : 0.f;
          C[(long long)row * sl.ldc + col] = v;
        }
      }
    }
  }
}

}  // namespace

void gemm_f32(const GemmParams& p0, GemmKind kind, int epi, int batch, hipStream_t st) {
  if (p0.M <= 0 || p0.N <= 0) return;
  GemmParams p = p0;
  int S = 1;
  if (p.splits > 1 && epi == EPI_STORE && p.ws != nullptr && p.K > 0 && p.Cp == nullptr) {
    const int kt = (p.K + BK - 1) / BK;
    p.kchunk = (kt + p.splits - 1) / p.splits * BK;
    S = (p.K + p.kchunk - 1) / p.kchunk;
  }
  p.splits = S;
  if (S == 1) p.kchunk = p.K;
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, batch * S);
  dim3 block(NTH);
  switch (kind) {
    case GEMM_NN:
      if (epi == EPI_BIAS_RELU)
        hipLaunchKernelGGL((gemm_f32_kernel<false, false, EPI_BIAS_RELU>), grid, block, 0, st, p);
      else
        hipLaunchKernelGGL((gemm_f32_kernel<false, false, EPI_STORE>), grid, block, 0, st, p);
      break;
    case GEMM_NT:
      if (epi == EPI_RELU_MASK)
        hipLaunchKernelGGL((gemm_f32_kernel<false, true, EPI_RELU_MASK>), grid, block, 0, st, p);
      else if (epi == EPI_BIAS_RELU)
        hipLaunchKernelGGL((gemm_f32_kernel<false, true, EPI_BIAS_RELU>), grid, block, 0, st, p);
      else
        hipLaunchKernelGGL((gemm_f32_kernel<false, true, EPI_STORE>), grid, block, 0, st, p);
      break;
    case GEMM_TN:
      hipLaunchKernelGGL((gemm_f32_kernel<true, false, EPI_STORE>), grid, block, 0, st, p);
      break;
  }
  if (S > 1) splitk_reduce(p, batch, S, st);
}

}  // namespace mtsac
