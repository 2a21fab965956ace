// gemm_x3.hip -- fp32-accurate GEMM on bf16 MFMA by 3-way operand splitting (gfx950).
//
// Same contract as gemm_f32.hip (GemmParams, NN / NT / TN, fused epilogues) but the
// products run on v_mfma_f32_32x32x16_bf16 (16x the f32-MFMA rate):
//   x = x_h + x_m + x_l  exactly, x_h = bf16_rn(x), x_m = bf16_rn(x - x_h), x_l = bf16_rn(x - x_h - x_m)
//   (each remainder is exact in fp32; 3 x 8 significant bits cover fp32's 24)
//   a.b ~= a_h b_h + a_h b_m + a_m b_h + a_h b_l + a_l b_h + a_m b_m
// Each bf16 x bf16 product is exact in fp32 and is accumulated in fp32; the dropped terms
// (a_m b_l, a_l b_m, a_l b_l) are <= 2^-23 relative, i.e. the error is that of an fp32 GEMM
// (tests/test_gpu_kernels.py measures it against float64).  6 bf16 MFMAs per k-slice cost
// 6/16 of the f32-MFMA time for the same work.
//
// Tile 128x128 per 256-thread workgroup, BK = 32, 2x2 waves each owning 2x2 32x32
// accumulators.  fp32 tiles are loaded to registers with the next K-tile in flight, split
// into three bf16 planes and stored k-contiguous in LDS ([plane][row][k], rows padded to
// 80 B so the MFMA operand reads -- one ds_read_b128 per lane -- are bank-conflict free).
#include "gemm_common.h"

namespace mtsac {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 32;
constexpr int NTH = 256;
constexpr int RS = 40;                  // LDS row stride in bf16 (80 B)
constexpr int PLANE = 128 * RS;         // one bf16 plane of a 128 x 32 operand tile
constexpr int OPER = 3 * PLANE;         // three planes

__device__ inline void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// Operand tile loader.  KCONT: source stored [rows][K] (k contiguous); else [K][rows].
// Each thread owns 4 rows x 4 k (transposing) or 1 row x 4 k repeated 4x (k-contiguous);
// either way it stores 4 x (3 planes x 4 bf16 = 8 B) into the [plane][row][k] image.
template <bool KCONT>
struct Loader {
  __device__ static inline void load(const float* __restrict__ base, int ld, int r0, int nrows, int k0, int K,
                                     float4 (&v)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KCONT) {
        const int kq = t & 7, r = (t >> 3) + 32 * i;
        const int row = r0 + r, k = k0 + 4 * kq;
        if (row < nrows && k < K) x = *reinterpret_cast<const float4*>(base + (long long)row * ld + k);
      } else {
        // kq fastest across lanes: 8 lanes x 16 B = 128 B per source row, and the LDS stores of
        // 16 consecutive lanes (kq 0-7, two rows 80 B apart) cover all 32 banks exactly once
        const int kq = t & 7, rq = t >> 3;
        const int k = k0 + 4 * kq + i, row = r0 + 4 * rq;
        if (k < K && row < nrows) x = *reinterpret_cast<const float4*>(base + (long long)k * ld + row);
      }
      v[i] = x;
    }
  }

  __device__ static inline void store(__bf16* __restrict__ lds, const float4 (&v)[4], int dbg) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row, kc;
      float e[4];
      if (KCONT) {
        row = (t >> 3) + 32 * i;
        kc = 4 * (t & 7);
        e[0] = v[i].x; e[1] = v[i].y; e[2] = v[i].z; e[3] = v[i].w;
      } else {  // 4x4 transpose in registers: row 4rq+i gets k = 4kq..4kq+3
        row = 4 * (t >> 3) + i;
        kc = 4 * (t & 7);
        const float* c0 = &v[0].x;
        const float* c1 = &v[1].x;
        const float* c2 = &v[2].x;
        const float* c3 = &v[3].x;
        e[0] = c0[i]; e[1] = c1[i]; e[2] = c2[i]; e[3] = c3[i];
      }
      bf16x4 h, m, l;
      if (dbg & 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) h[j] = m[j] = l[j] = (__bf16)e[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 a, b, c;
          split3(e[j], a, b, c);
          h[j] = a;
          m[j] = b;
          l[j] = c;
        }
      }
      __bf16* p = lds + row * RS + kc;
      *reinterpret_cast<bf16x4*>(p) = h;
      *reinterpret_cast<bf16x4*>(p + PLANE) = m;
      *reinterpret_cast<bf16x4*>(p + 2 * PLANE) = l;
    }
  }
};

template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(NTH, 2) void gemm_x3_kernel(GemmParams p, int dbg) {
  // A: TA ? [K][M] : [M][K] (k contiguous);  B: TB ? [N][K] (k contiguous) : [K][N]
  using LA = Loader<!TA>;
  using LB = Loader<TB>;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * OPER];
  __bf16* As = smem;
  __bf16* Bs = smem + OPER;

  const GemmSlice sl = gemm_slice<TA, TB>(p);
  const int z = sl.z;
  const float* __restrict__ A = sl.A;
  const float* __restrict__ B = sl.B;
  float* __restrict__ C = sl.C;
  const int K = sl.K;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int t = threadIdx.x;
  const int wave = t >> 6, lane = t & 63;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int lr = lane & 31, lh = lane >> 5;

  const bool do_db = (EPI == EPI_STORE) && !TB && sl.db != nullptr && blockIdx.x == 0;
  float dbacc = 0.f;
  f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};

  float4 ra[4], rb[4];
  const int nk = (K + BK - 1) / BK;
  LA::load(A, p.lda, m0, p.M, 0, K, ra);
  LB::load(B, p.ldb, n0, p.N, 0, K, rb);
  LA::store(As, ra, 0);
  LB::store(Bs, rb, 0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = (kt + 1) < nk;
    if (more && !(dbg & 1)) {
      LA::load(A, p.lda, m0, p.M, (kt + 1) * BK, K, ra);
      LB::load(B, p.ldb, n0, p.N, (kt + 1) * BK, K, rb);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int ko = 16 * ks + 8 * lh;
      bf16x8 a[2][3], b[2][3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          a[i][q] = *reinterpret_cast<const bf16x8*>(As + q * PLANE + (wm + 32 * i + lr) * RS + ko);
          b[i][q] = *reinterpret_cast<const bf16x8*>(Bs + q * PLANE + (wn + 32 * i + lr) * RS + ko);
        }
      }
#define X3_TILE(ACC, I, J)                                                                  \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[I][1], b[J][1], ACC, 0, 0, 0);           \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[I][0], b[J][2], ACC, 0, 0, 0);           \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[I][2], b[J][0], ACC, 0, 0, 0);           \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[I][0], b[J][1], ACC, 0, 0, 0);           \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[I][1], b[J][0], ACC, 0, 0, 0);           \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[I][0], b[J][0], ACC, 0, 0, 0);
      if (dbg & 2) {
        acc00[0] += (float)a[0][0][0] + (float)a[1][1][1] + (float)a[0][2][2];
        acc01[0] += (float)b[0][0][0] + (float)b[1][1][1] + (float)b[0][2][2];
        acc10[0] += (float)a[1][0][0] + (float)a[0][1][1] + (float)a[1][2][2];
        acc11[0] += (float)b[1][0][0] + (float)b[0][1][1] + (float)b[1][2][2];
        continue;
      }
      X3_TILE(acc00, 0, 0)
      X3_TILE(acc01, 0, 1)
      X3_TILE(acc10, 1, 0)
      X3_TILE(acc11, 1, 1)
#undef X3_TILE
    }
    if (do_db) {  // column sums of the B tile (= dZ rows of this K-tile): h + m + l is exact
      const int col = t & 127, half = t >> 7;
      const __bf16* q0 = Bs + col * RS + 16 * half;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        dbacc += ((float)q0[r] + (float)q0[PLANE + r]) + (float)q0[2 * PLANE + r];
    }
    __syncthreads();
    if (more) {
      LA::store(As, ra, dbg);
      LB::store(Bs, rb, dbg);
      __syncthreads();
    }
  }

  if (do_db) {
    float* red = reinterpret_cast<float*>(smem);
    const int col = t & 127, half = t >> 7;
    if (half == 1) red[col] = dbacc;
    __syncthreads();
    if (half == 0 && n0 + col < p.N) sl.db[n0 + col] = dbacc + red[col];
  }

  TileOut o{};
  o.C = C;
  o.ldc = sl.ldc;
  o.bias = (EPI == EPI_BIAS_RELU) ? p.bias + z * p.sBias : nullptr;
  o.mask = (EPI == EPI_RELU_MASK) ? p.mask + z * p.sMask : nullptr;
  o.ldm = p.ldm;
  o.Cp = p.Cp ? p.Cp + z * p.sCp : nullptr;
  o.ldcp = p.ldcp;
  o.pC = p.pC;
  o.M = p.M;
  o.N = p.N;
  o.vec = (p.N % 4 == 0) && (sl.ldc % 4 == 0) && (EPI != EPI_RELU_MASK || p.ldm % 4 == 0) &&
          (!p.Cp || p.ldcp % 4 == 0);
  __syncthreads();  // operand tiles (and the db scratch) are dead: reuse LDS as store scratch
  float* scr = reinterpret_cast<float*>(smem) + wave * (32 * 36);
  float omx = 0.f;  // (split2h maxima: the fp32-operand kernel writes split3 planes only)
  store_tile32<EPI>(acc00, scr, lane, m0 + wm, n0 + wn, o, omx);
  store_tile32<EPI>(acc01, scr, lane, m0 + wm, n0 + wn + 32, o, omx);
  store_tile32<EPI>(acc10, scr, lane, m0 + wm + 32, n0 + wn, o, omx);
  store_tile32<EPI>(acc11, scr, lane, m0 + wm + 32, n0 + wn + 32, o, omx);
}

}  // namespace

int g_x3_dbg = 0;

void gemm_x3(const GemmParams& p0, GemmKind kind, int epi, int batch, hipStream_t st) {
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
        hipLaunchKernelGGL((gemm_x3_kernel<false, false, EPI_BIAS_RELU>), grid, block, 0, st, p, g_x3_dbg);
      else
        hipLaunchKernelGGL((gemm_x3_kernel<false, false, EPI_STORE>), grid, block, 0, st, p, g_x3_dbg);
      break;
    case GEMM_NT:
      if (epi == EPI_RELU_MASK)
        hipLaunchKernelGGL((gemm_x3_kernel<false, true, EPI_RELU_MASK>), grid, block, 0, st, p, g_x3_dbg);
      else if (epi == EPI_BIAS_RELU)
        hipLaunchKernelGGL((gemm_x3_kernel<false, true, EPI_BIAS_RELU>), grid, block, 0, st, p, g_x3_dbg);
      else
        hipLaunchKernelGGL((gemm_x3_kernel<false, true, EPI_STORE>), grid, block, 0, st, p, g_x3_dbg);
      break;
    case GEMM_TN:
      hipLaunchKernelGGL((gemm_x3_kernel<true, false, EPI_STORE>), grid, block, 0, st, p, g_x3_dbg);
      break;
  }
  if (S > 1) splitk_reduce(p, batch, S, st);
}

}  // namespace mtsac
