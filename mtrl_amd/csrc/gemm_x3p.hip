// gemm_x3p.hip -- fp32-accurate GEMM on PRE-SPLIT bf16 planes (gfx950).
//
// Operands arrive as three bf16 planes each (x = x_h + x_m + x_l exactly, see gemm_x3.hip),
// k-contiguous: A planes [3][M][lda], B planes [3][N][ldb] (C = A . B^T), K padded with
// zeros to a multiple of 32 in both.  So the main loop has no VALU at all:
//   * global -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane), 3-stage ring,
//     counted vmcnt + raw s_barrier (one barrier per 32-deep K-step, loads for step k+2
//     in flight while step k computes);
//   * LDS image [row][4 x 16 B] per plane, chunk XOR-swizzled by (row >> 2) & 3 -- done on
//     the SOURCE address because the DMA writes lane-linearly -- so the MFMA operand
//     reads (one ds_read_b128 per lane) are bank-conflict free;
//   * 6 x v_mfma_f32_32x32x16_bf16 per 32x32 tile and 16-deep k-slice (m*m, h*l, l*h, h*m,
//     m*h, h*h; small terms first), fp32 accumulation.
// Tile 128x128 per 256-thread workgroup (2x2 waves of 64x64), 144 KiB LDS, one block per CU.
// Epilogue: fp32 C with bias+ReLU / ReLU-mask / plain, optionally also the split planes of
// C (natural layout) for the next GEMM.
#include "kernels.h"

namespace mtsac {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int BK = 32;
constexpr int ROWB = BK * 2;  // 64 B per row per plane

__device__ inline int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// Tile geometry: BM x BN per workgroup, WM x WN waves, each wave (BM/WM) x (BN/WN) made of
// 32x32 MFMA tiles; STAGES-deep LDS ring of [3 planes][rows][64 B] images.
template <int BM_, int BN_, int WM_, int WN_, int STAGES_>
struct Geo {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, STAGES = STAGES_;
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  static constexpr int TI = BM / WM / 32, TJ = BN / WN / 32;
  static constexpr int PLANE_A = BM * ROWB, PLANE_B = BN * ROWB;
  static constexpr int OPER_A = 3 * PLANE_A, OPER_B = 3 * PLANE_B;
  static constexpr int STAGE = OPER_A + OPER_B;
  static constexpr int LDS = STAGES * STAGE;
  static constexpr int DMA_A = 3 * BM / 16, DMA_B = 3 * BN / 16;  // 1 KiB wave-instructions
  static constexpr int DMA_PER_WAVE = (DMA_A + DMA_B) / NW;
  static_assert((DMA_A + DMA_B) % NW == 0, "DMA split");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// Issue the LDS-DMA loads of one operand tile (3 planes x ROWS x 32 k) into `lds`: the
// wave-instructions j = first, first + stride, ... of the 3*ROWS/16 needed.
template <int ROWS>
__device__ inline void dma_tile(const __bf16* __restrict__ base, long long ld, long long plane_stride, int r0,
                                int nrows, int k0, char* lds, int first, int stride) {
  constexpr int NJ = 3 * ROWS / 16, PER_PLANE = ROWS / 16;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = first; j < NJ; j += stride) {
    const int q = j / PER_PLANE;              // plane
    const int rb = (j % PER_PLANE) * 16;      // first row of this instruction
    const int row = rb + (lane >> 2);         // physical row written by this lane
    const int logical = swz(row, lane & 3);   // chunk to fetch so the image comes out swizzled
    int grow = r0 + row;
    grow = grow < nrows ? grow : nrows - 1;   // clamp: rows past the edge feed discarded outputs
    const __bf16* src = base + q * plane_stride + (long long)grow * ld + k0 + 8 * logical;
    char* dst = lds + q * (ROWS * ROWB) + rb * ROWB;
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

template <class G>
__device__ inline void dma_stage(const SplitGemmParams& p, const __bf16* A, const __bf16* B, int m0, int n0, int k0,
                                 char* st, int wave) {
  // A's and B's wave-instructions are dealt round-robin over all waves
  dma_tile<G::BM>(A, p.lda, p.pA, m0, p.M, k0, st, wave, G::NW);
  const int fb = (G::NW - (G::DMA_A % G::NW) + wave) % G::NW;
  dma_tile<G::BN>(B, p.ldb, p.pB, n0, p.N, k0, st + G::OPER_A, fb, G::NW);
}

template <class G, int EPI, bool PLANES_OUT>
__global__ __launch_bounds__(G::NTH, 1) void gemm_x3p_kernel(SplitGemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  char* lds = smem;
  const int z = blockIdx.z;
  const __bf16* __restrict__ A = p.A + z * p.sA;
  const __bf16* __restrict__ B = p.B + z * p.sB;
  const int m0 = blockIdx.x * G::BM, n0 = blockIdx.y * G::BN;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (wave % G::WM) * (G::BM / G::WM), wn = (wave / G::WM) * (G::BN / G::WN);
  const int lr = lane & 31, lh = lane >> 5;
  const int nk = p.K / BK;  // K is padded to a multiple of BK

  f32x16 acc[G::TI][G::TJ];
#pragma unroll
  for (int i = 0; i < G::TI; ++i)
#pragma unroll
    for (int j = 0; j < G::TJ; ++j) acc[i][j] = f32x16{0};

  // prologue: the first STAGES-1 stages in flight
#pragma unroll
  for (int s = 0; s < G::STAGES - 1; ++s)
    if (s < nk) dma_stage<G>(p, A, B, m0, n0, s * BK, lds + s * G::STAGE, wave);

  for (int kt = 0; kt < nk; ++kt) {
    // retire stage kt (younger stages may stay in flight), then one barrier: every wave's
    // stage-kt data has landed and every wave is done reading the buffer about to be refilled
    const int younger = min(G::STAGES - 2, nk - 1 - kt);
    if (younger >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::DMA_PER_WAVE) : "memory");
    else if (younger == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::DMA_PER_WAVE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + G::STAGES - 1 < nk && !(p.dbg & 1))
      dma_stage<G>(p, A, B, m0, n0, (kt + G::STAGES - 1) * BK, lds + ((kt + G::STAGES - 1) % G::STAGES) * G::STAGE,
                   wave);
    const char* cur = lds + (kt % G::STAGES) * G::STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int chunk = 2 * ks + lh;
      bf16x8 a[G::TI][3], b[G::TJ][3];
#pragma unroll
      for (int i = 0; i < G::TI; ++i) {
        const int r = wm + 32 * i + lr;
        const int o = r * ROWB + 16 * swz(r, chunk);
#pragma unroll
        for (int q = 0; q < 3; ++q) a[i][q] = *reinterpret_cast<const bf16x8*>(cur + q * G::PLANE_A + o);
      }
#pragma unroll
      for (int j = 0; j < G::TJ; ++j) {
        const int r = wn + 32 * j + lr;
        const int o = r * ROWB + 16 * swz(r, chunk);
#pragma unroll
        for (int q = 0; q < 3; ++q)
          b[j][q] = *reinterpret_cast<const bf16x8*>(cur + G::OPER_A + q * G::PLANE_B + o);
      }
      if (p.dbg & 2) {
#pragma unroll
        for (int i = 0; i < G::TI; ++i)
#pragma unroll
          for (int j = 0; j < G::TJ; ++j) acc[i][j][0] += (float)a[i][0][0] + (float)b[j][2][7];
        continue;
      }
#pragma unroll
      for (int i = 0; i < G::TI; ++i)
#pragma unroll
        for (int j = 0; j < G::TJ; ++j) {
          f32x16 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);  // m*m
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);  // h*l
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);  // l*h
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);  // h*m
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);  // m*h
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);  // h*h
          acc[i][j] = c;
        }
    }
  }

  float* __restrict__ C = p.C ? p.C + z * p.sC : nullptr;
  const float* __restrict__ bias = (EPI == EPI_BIAS_RELU) ? p.bias + z * p.sBias : nullptr;
  const float* __restrict__ mask = (EPI == EPI_RELU_MASK) ? p.mask + z * p.sMask : nullptr;
#pragma unroll
  for (int j = 0; j < G::TJ; ++j) {
    const int col = n0 + wn + 32 * j + lr;
    const bool colok = col < p.N;
    const float bv = (EPI == EPI_BIAS_RELU && colok) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < G::TI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < p.M && colok) {
          float v = acc[i][j][r];
          if (EPI == EPI_BIAS_RELU) v = fmaxf(v + bv, 0.f);
          if (EPI == EPI_RELU_MASK) v = (mask[(long long)row * p.ldm + col] > 0.f) ? v : 0.f;
          if (C) C[(long long)row * p.ldc + col] = v;
          if (PLANES_OUT) {
            __bf16* cp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
            const __bf16 h = (__bf16)v;
            const float r1 = v - (float)h;
            const __bf16 m = (__bf16)r1;
            cp[0] = h;
            cp[p.pC] = m;
            cp[2 * p.pC] = (__bf16)(r1 - (float)m);
          }
        }
      }
    }
  }
}

using GeoSmall = Geo<128, 128, 2, 2, 3>;  // 4 waves, 144 KiB
using GeoWide = Geo<256, 128, 4, 2, 2>;   // 8 waves, 144 KiB

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
      o = (long long)orow * s.ldo + ocol;
    } else {
      v = tile[a][b];
      const int orow = r0 + a, ocol = c0 + b;
      if (orow >= s.out_rows || ocol >= s.out_cols) continue;
      o = (long long)orow * s.ldo + ocol;
    }
    const __bf16 h = (__bf16)v;
    const float r1 = v - (float)h;
    const __bf16 m = (__bf16)r1;
    out[o] = h;
    out[o + s.po] = m;
    out[o + 2 * s.po] = (__bf16)(r1 - (float)m);
  }
}

// db[z][n] = sum over rows of x[z][rows][n] in two deterministic passes
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x, int rows, int cols, int ld,
                                                             long long sx, int chunks, float* __restrict__ part) {
  const int z = blockIdx.z, c = blockIdx.x * 256 + threadIdx.x, ch = blockIdx.y;
  if (c >= cols) return;
  const int per = (rows + chunks - 1) / chunks;
  const int r0 = ch * per, r1 = min(rows, r0 + per);
  const float* xp = x + z * sx;
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += xp[(long long)r * ld + c];
  part[((long long)z * chunks + ch) * cols + c] = s;
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int cols, int chunks,
                                                           float* __restrict__ db, long long sdb) {
  const int z = blockIdx.z, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int ch = 0; ch < chunks; ++ch) s += part[((long long)z * chunks + ch) * cols + c];
  db[z * sdb + c] = s;
}

}  // namespace

template <class G>
static void launch_x3p(const SplitGemmParams& p, int epi, int batch, hipStream_t st) {
  dim3 grid((p.M + G::BM - 1) / G::BM, (p.N + G::BN - 1) / G::BN, batch);
  const bool planes = p.Cp != nullptr;
  if (epi == EPI_BIAS_RELU) {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, EPI_BIAS_RELU, true>), grid, dim3(G::NTH), 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, EPI_BIAS_RELU, false>), grid, dim3(G::NTH), 0, st, p);
  } else if (epi == EPI_RELU_MASK) {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, EPI_RELU_MASK, true>), grid, dim3(G::NTH), 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, EPI_RELU_MASK, false>), grid, dim3(G::NTH), 0, st, p);
  } else {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, EPI_STORE, true>), grid, dim3(G::NTH), 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, EPI_STORE, false>), grid, dim3(G::NTH), 0, st, p);
  }
}

int g_x3p_geo = 1;
int g_x3p_dbg = 0;  // 0: 128x128 / 4 waves, 1: 256x128 / 8 waves

void gemm_x3p(const SplitGemmParams& p, int epi, int batch, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return;
  SplitGemmParams q = p;
  q.dbg |= g_x3p_dbg;
  if (g_x3p_geo == 0)
    launch_x3p<GeoSmall>(q, epi, batch, st);
  else
    launch_x3p<GeoWide>(q, epi, batch, st);
}

void split_planes(const SplitParams& s, bool transpose, int batch, hipStream_t st) {
  dim3 grid((s.rows + 63) / 64, (s.cols + 63) / 64, batch);
  if (transpose)
    hipLaunchKernelGGL(split_kernel<true>, grid, dim3(256), 0, st, s);
  else
    hipLaunchKernelGGL(split_kernel<false>, grid, dim3(256), 0, st, s);
}

void colsum(const float* x, int rows, int cols, int ld, long long sx, int batch, float* part, float* db,
            long long sdb, hipStream_t st) {
  const int chunks = 16;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((cols + 255) / 256, chunks, batch), dim3(256), 0, st, x, rows, cols,
                     ld, sx, chunks, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 255) / 256, 1, batch), dim3(256), 0, st, part, cols, chunks, db,
                     sdb);
}

}  // namespace mtsac
