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

#include "gemm_common.h"

namespace mtsac {

typedef f32x16_t f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int BK = 32;  // K granule of the operands (split-K slices, padding); K-steps are 16 or 32

typedef __attribute__((address_space(3))) void lds_void;

__device__ inline void glds16(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)dst, 16, 0, 0);
}

// One operand's image of a K-step: R rows (M or N) x KS k, three planes.
template <int R, bool KM, int KS>
struct Oper {
  static constexpr int PLANE = R * KS * 2;  // bytes per plane
  static constexpr int BYTES = 3 * PLANE;
  static constexpr int NJ = 3 * PLANE / 1024;  // 1-KiB wave-instructions per stage
  static constexpr int ROWB = KM ? 2 * R : 2 * KS;
  static constexpr int RPI = 1024 / ROWB;   // image rows per wave-instruction
  static constexpr int LPR = ROWB / 16;     // lanes per image row
  static constexpr int PER_PLANE = NJ / 3;
  static_assert(!KM || LPR >= 16, "k-major swizzle needs >= 16 chunks per row");

  // physical 16-B chunk of logical chunk c in image row irow (conflict-free reads, see header)
  __device__ static inline int pchunk(int irow, int c) {
    if (KM) return c ^ (4 * (irow & 3));
    return KS == 32 ? (c ^ ((irow >> 2) & 3)) : (c ^ ((irow >> 3) & 1));
  }

  // issue wave-instructions first, first + stride, ... (< NJ) of the stage at k0
  __device__ static inline void dma(const __bf16* __restrict__ base, long long ld, long long ps, int r0, int nrows,
                                    int k0, char* lds, int first, int stride) {
#pragma unroll
    for (int j = first; j < NJ; j += stride) dma_one(base, ld, ps, r0, nrows, k0, lds, j);
  }

  // wave-instruction j (< NJ) of the stage at k0
  __device__ static inline void dma_one(const __bf16* __restrict__ base, long long ld, long long ps, int r0, int nrows,
                                        int k0, char* lds, int j) {
    const int lane = threadIdx.x & 63;
    {
      const int q = j / PER_PLANE;
      const int ib = (j % PER_PLANE) * RPI;  // first image row of the instruction
      const int irow = ib + lane / LPR;
      const int c = pchunk(irow, lane % LPR);  // logical chunk this lane fetches (XOR is an involution)
      const __bf16* src;
      if (KM) {  // image row = k, chunk = 8 columns
        int col = r0 + 8 * c;
        const int last = ((nrows + 7) & ~7) - 8;
        col = col < last ? col : last;  // columns past the edge feed discarded outputs
        src = base + q * ps + (long long)(k0 + irow) * ld + col;
      } else {   // image row = row, chunk = 8 k
        int row = r0 + irow;
        row = row < nrows ? row : nrows - 1;
        src = base + q * ps + (long long)row * ld + k0 + 8 * c;
      }
      glds16(src, lds + q * PLANE + ib * ROWB);
    }
  }

  // MFMA fragment of plane q: 8 bf16 = k 16ks + 8h .. +7 of row rb + (lane & 31)
  __device__ static inline bf16x8 frag(const char* lds, int q, int rb, int ks, int lane) {
    const char* pl = lds + q * PLANE;
    if (!KM) {
      const int r = rb + (lane & 31);
      const int o = r * ROWB + 16 * pchunk(r, (KS / 8 == 4 ? 2 * ks : 0) + (lane >> 5));
      return *reinterpret_cast<const bf16x8*>(pl + o);
    } else {
      // ds_read_b64_tr_b16: 16-lane group G reads a 4 k x 16 column block; lane 4qq+p gives the
      // address of k-row qq, columns 4p..4p+3; lane i receives column i (= its MFMA row).
      const int G = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
      const int m = rb + 16 * (G & 1) + 4 * p;
      const int c = m >> 3, inb = 8 * (p & 1);
      const int k0 = 16 * ks + 8 * (G >> 1) + qq;
      const int o0 = k0 * ROWB + 16 * pchunk(k0, c) + inb;
      const int o1 = (k0 + 4) * ROWB + 16 * pchunk(k0 + 4, c) + inb;
      const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(pl + o0));
      const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(pl + o1));
      const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

// Tile geometry: BM x BN per workgroup, WM x WN waves, each wave (BM/WM) x (BN/WN) made of
// 32x32 MFMA tiles; STAGES-deep LDS ring.
// TAG only separates kernel symbols (e.g. input-layer launches in profiles)
template <int BM_, int BN_, int WM_, int WN_, int STAGES_, int KS_, int TAG = 0>
struct Geo {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, STAGES = STAGES_, KS = KS_;
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  static constexpr int TI = BM / WM / 32, TJ = BN / WN / 32;
};

template <class G, bool AKM, bool BKM, int EPI, bool PLANES_OUT>
__global__ __launch_bounds__(G::NTH, 1) void gemm_x3p_kernel(SplitGemmParams p) {
  using OA = Oper<G::BM, AKM, G::KS>;
  using OB = Oper<G::BN, BKM, G::KS>;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  // the stage's wave-instructions are dealt round robin: waves < DMA_X issue one more
  constexpr int DMA_LO = (OA::NJ + OB::NJ) / G::NW, DMA_X = (OA::NJ + OB::NJ) % G::NW;
  static_assert(G::STAGES * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[G::STAGES * STAGE];
  char* lds = smem;

  // XCD-aware tile order: the grid is 1-D; consecutive workgroups land on different XCDs
  // (round robin), so hand each XCD a contiguous run of tiles, N-tile fastest -- the
  // workgroups resident on one XCD then share a few A row-blocks and every B column-block
  // through its L2.
  const int ny = (p.N + G::BN - 1) / G::BN, nx = (p.M + G::BM - 1) / G::BM;
  int tile = blockIdx.x;
  if (!(p.dbg & 4)) {
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = tile % 8;
    tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + tile / 8;
  }
  const int by = tile % ny, bx = (tile / ny) % nx;
  const int S = p.splits > 1 ? p.splits : 1;
  const int zz = tile / (ny * nx), z = zz / S, sp = zz - z * S;
  const int kbeg = sp * p.kchunk;
  const int Kl = S > 1 ? min(p.kchunk, p.K - kbeg) : p.K;
  const __bf16* __restrict__ A = p.A + z * p.sA + (AKM ? (long long)kbeg * p.lda : (long long)kbeg);
  const __bf16* __restrict__ B = p.B + z * p.sB + (BKM ? (long long)kbeg * p.ldb : (long long)kbeg);
  const int m0 = bx * G::BM, n0 = by * G::BN;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (wave % G::WM) * (G::BM / G::WM), wn = (wave / G::WM) * (G::BN / G::WN);
  const int lr = lane & 31, lh = lane >> 5;
  const int nk = Kl / G::KS;
  const int fb = (G::NW - (OA::NJ % G::NW) + wave) % G::NW;  // B's instructions continue the round robin

  auto stage = [&](int s, int k0) {
    char* st = lds + s * STAGE;
    OA::dma(A, p.lda, p.pA, m0, p.M, k0, st, wave, G::NW);
    OB::dma(B, p.ldb, p.pB, n0, p.N, k0, st + OA::BYTES, fb, G::NW);
  };
  // the wave's q-th wave-instruction of a stage (same dealing as stage(): global index
  // wave + q * NW, A's instructions first)
  auto piece = [&](int s, int k0, int q) {
    char* st = lds + s * STAGE;
    const int jg = wave + q * G::NW;
    if (jg < OA::NJ)
      OA::dma_one(A, p.lda, p.pA, m0, p.M, k0, st, jg);
    else if (jg - OA::NJ < OB::NJ)
      OB::dma_one(B, p.ldb, p.pB, n0, p.N, k0, st + OA::BYTES, jg - OA::NJ);
  };
  (void)fb;
  constexpr int PIECES = DMA_LO + (DMA_X ? 1 : 0);          // per wave and stage (the last maybe empty)
  constexpr int SLOTS = (G::KS / 16) * G::TI * G::TJ;        // MFMA groups per K-step

  f32x16 acc[G::TI][G::TJ];
#pragma unroll
  for (int i = 0; i < G::TI; ++i)
#pragma unroll
    for (int j = 0; j < G::TJ; ++j) acc[i][j] = f32x16{0};

#pragma unroll
  for (int s = 0; s < G::STAGES - 1; ++s)
    if (s < nk) stage(s, s * G::KS);

  for (int kt = 0; kt < nk; ++kt) {
    // retire stage kt (younger stages may stay in flight), then one barrier: every wave's
    // stage-kt data has landed and every wave is done reading the buffer about to be refilled
    const int younger = min(G::STAGES - 2, nk - 1 - kt);
    const bool more = DMA_X != 0 && wave < DMA_X;
    if (younger >= 3) {
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DMA_LO + 1)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * DMA_LO) : "memory");
    } else if (younger == 2) {
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DMA_LO + 1)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DMA_LO) : "memory");
    } else if (younger == 1) {
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_LO + 1) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_LO) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // the refill of the slot read at kt-1 is spread over this K-step's MFMA groups (p.dbg & 8:
    // all issued up front)
    const bool refill = kt + G::STAGES - 1 < nk && !(p.dbg & 1);
    const int rs = (kt + G::STAGES - 1) % G::STAGES, rk = (kt + G::STAGES - 1) * G::KS;
    if (refill && (p.dbg & 8)) stage(rs, rk);
    const bool spread = refill && !(p.dbg & 8);
    const char* cur = lds + (kt % G::STAGES) * STAGE;
#pragma unroll
    for (int ks = 0; ks < G::KS / 16; ++ks) {
      bf16x8 a[G::TI][3], b[G::TJ][3];
#pragma unroll
      for (int i = 0; i < G::TI; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) a[i][q] = OA::frag(cur, q, wm + 32 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < G::TJ; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) b[j][q] = OB::frag(cur + OA::BYTES, q, wn + 32 * j, ks, lane);
      if (p.dbg & 2) {
#pragma unroll
        for (int i = 0; i < G::TI; ++i)
#pragma unroll
          for (int j = 0; j < G::TJ; ++j) acc[i][j][0] += (float)a[i][0][0] + (float)b[j][2][7];
        if (spread && ks == 0)
#pragma unroll
          for (int q = 0; q < PIECES; ++q) piece(rs, rk, q);
        continue;
      }
#pragma unroll
      for (int i = 0; i < G::TI; ++i)
#pragma unroll
        for (int j = 0; j < G::TJ; ++j) {
          const int slot = (ks * G::TI + i) * G::TJ + j;
          if (spread) {
#pragma unroll
            for (int q = slot * PIECES / SLOTS; q < (slot + 1) * PIECES / SLOTS; ++q) piece(rs, rk, q);
          }
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

  TileOut o{};
  if (S > 1) {
    o.C = p.ws + (long long)zz * p.M * p.N;
    o.ldc = p.N;
  } else {
    o.C = p.C ? p.C + z * p.sC : nullptr;
    o.ldc = p.ldc;
  }
  o.bias = (EPI == EPI_BIAS_RELU) ? p.bias + z * p.sBias : nullptr;
  o.mask = (EPI == EPI_RELU_MASK) ? p.mask + z * p.sMask : nullptr;
  o.ldm = p.ldm;
  o.Cp = PLANES_OUT ? p.Cp + z * p.sCp : nullptr;
  o.ldcp = p.ldcp;
  o.pC = p.pC;
  o.M = p.M;
  o.N = p.N;
  o.vec = (p.N % 4 == 0) && (o.ldc % 4 == 0) && (EPI != EPI_RELU_MASK || p.ldm % 4 == 0) &&
          (!PLANES_OUT || p.ldcp % 4 == 0);
  __builtin_amdgcn_s_barrier();  // every wave is done with the ring: reuse it as scratch
  float* scr = reinterpret_cast<float*>(smem) + wave * (32 * 36);
#pragma unroll
  for (int i = 0; i < G::TI; ++i)
#pragma unroll
    for (int j = 0; j < G::TJ; ++j) store_tile32<EPI>(acc[i][j], scr, lane, m0 + wm + 32 * i, n0 + wn + 32 * j, o);
}

using GeoSmall = Geo<128, 128, 2, 2, 3, 32>;   // 4 waves, 3 x 48 KiB
using GeoWide = Geo<256, 128, 4, 2, 2, 32>;    // 8 waves, 2 x 72 KiB
using GeoWide16 = Geo<256, 128, 4, 2, 4, 16>;  // 8 waves, 4 x 36 KiB
using GeoBig16 = Geo<256, 256, 2, 4, 3, 16>;   // 8 waves of 128 x 64, 3 x 48 KiB
using GeoSmall16 = Geo<128, 128, 2, 2, 3, 16>;  // 4 waves, 3 x 24 KiB: two workgroups per CU
using GeoBig16In = Geo<256, 256, 2, 4, 3, 16, 1>;  // GeoBig16 for input-layer launches (own symbol)

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

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int cols, int chunks,
                                                           float* __restrict__ db, long long sdb) {
  const int z = blockIdx.z, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int ch = 0; ch < chunks; ++ch) s += part[((long long)z * chunks + ch) * cols + c];
  db[z * sdb + c] = s;
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

template <class G, bool AKM, bool BKM>
static void launch_x3p(const SplitGemmParams& p, int epi, dim3 grid, hipStream_t st) {
  const bool planes = p.Cp != nullptr;
  const dim3 block(G::NTH);
  if (epi == EPI_BIAS_RELU) {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_BIAS_RELU, true>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_BIAS_RELU, false>), grid, block, 0, st, p);
  } else if (epi == EPI_RELU_MASK) {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_RELU_MASK, true>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_RELU_MASK, false>), grid, block, 0, st, p);
  } else {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_STORE, true>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_STORE, false>), grid, block, 0, st, p);
  }
}

template <class G>
static void launch_geo(const SplitGemmParams& p, int epi, int batch, hipStream_t st) {
  dim3 grid(((p.M + G::BM - 1) / G::BM) * ((p.N + G::BN - 1) / G::BN) * batch * (p.splits > 1 ? p.splits : 1));
  if (!p.a_kmajor && !p.b_kmajor)
    launch_x3p<G, false, false>(p, epi, grid, st);
  else if (p.a_kmajor && p.b_kmajor)
    launch_x3p<G, true, true>(p, epi, grid, st);
  else if (p.a_kmajor)
    launch_x3p<G, true, false>(p, epi, grid, st);
  else
    launch_x3p<G, false, true>(p, epi, grid, st);
}

int g_x3p_geo = -1;  // -1: by operand form; 0: 128x128 k32, 1: 256x128 k32, 2: 256x128 k16, 3: 256x256 k16
int g_x3p_dbg = 0;

// tile shape of a geometry id (see Geo aliases above)
static void geo_tile(int geo, int& bm, int& bn) {
  bm = (geo == 0 || geo == 4) ? 128 : 256;
  bn = geo == 3 ? 256 : 128;
}

// Auto geometry by size (measured, tools/x3p_bench.py): 256x256 tiles (least operand traffic
// per MFMA) when they give >= 192 workgroups or the form is the k-major weight gradient (split-K
// fills the chip there); else 256x128.  g_x3p_geo forces one (experiments).
static int pick_geo(int M, int N, int batch, bool kmajor) {
  if (g_x3p_geo >= 0) return g_x3p_geo;
  if (kmajor) return 3;
  const long long big = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  return big >= 192 ? 3 : 1;
}

int gemm_x3p_splits(int M, int N, int K, int batch, bool kmajor) {
  int bm, bn;
  geo_tile(pick_geo(M, N, batch, kmajor), bm, bn);
  const long long tiles = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch;
  if (tiles >= 192) return 1;
  int s = (int)((256 + tiles - 1) / tiles);
  s = std::min(s, kmajor ? 16 : 4);
  s = std::min(s, std::max(1, K / BK / 8));  // >= 8 K-granules per slice
  return std::max(s, 1);
}

long long gemm_x3p_ws_floats(int M, int N, int K, int batch, bool kmajor) {
  return gemm_ws_floats(M, N, batch, gemm_x3p_splits(M, N, K, batch, kmajor));
}

namespace {

// split-K finish: C = epi(sum_s ws[z*S+s]) (+ its planes), slices added in order
template <int EPI>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(SplitGemmParams p, int S, int batch) {
  const long long slab = (long long)p.M * p.N;
  const int n4 = p.N / 4;
  const long long per = (long long)p.M * n4;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= per * batch) return;
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
  if (EPI == EPI_RELU_MASK) {
    const float4 mk = *reinterpret_cast<const float4*>(p.mask + z * p.sMask + (long long)row * p.ldm + col);
    e[0] = mk.x > 0.f ? e[0] : 0.f; e[1] = mk.y > 0.f ? e[1] : 0.f;
    e[2] = mk.z > 0.f ? e[2] : 0.f; e[3] = mk.w > 0.f ? e[3] : 0.f;
  }
  if (p.C) *reinterpret_cast<float4*>(p.C + z * p.sC + (long long)row * p.ldc + col) = make_float4(e[0], e[1], e[2], e[3]);
  if (p.Cp) {
    bf16x4_t h, m, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __bf16 a, b, c;
      split3_dev(e[j], a, b, c);
      h[j] = a; m[j] = b; l[j] = c;
    }
    __bf16* cp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
    *reinterpret_cast<bf16x4_t*>(cp) = h;
    *reinterpret_cast<bf16x4_t*>(cp + p.pC) = m;
    *reinterpret_cast<bf16x4_t*>(cp + 2 * p.pC) = l;
  }
}

}  // namespace

void gemm_x3p(const SplitGemmParams& p0, int epi, int batch, hipStream_t st) {
  if (p0.M <= 0 || p0.N <= 0 || p0.K <= 0) return;
  SplitGemmParams p = p0;
  p.dbg |= g_x3p_dbg;
  const bool kmajor = p.a_kmajor && p.b_kmajor;
  if (p.splits < 0) p.splits = gemm_x3p_splits(p.M, p.N, p.K, batch, kmajor);  // auto
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
  switch (pick_geo(p.M, p.N, batch, kmajor)) {
    case 0: launch_geo<GeoSmall>(q, kepi, batch, st); break;
    case 2: launch_geo<GeoWide16>(q, kepi, batch, st); break;
    case 3:
      if (p.tag == 1)
        launch_geo<GeoBig16In>(q, kepi, batch, st);
      else
        launch_geo<GeoBig16>(q, kepi, batch, st);
      break;
    case 4: launch_geo<GeoSmall16>(q, kepi, batch, st); break;
    default: launch_geo<GeoWide>(q, kepi, batch, st); break;
  }
  if (S == 1) return;
  if (epi == EPI_STORE && !p.Cp) {
    GemmParams r{};
    r.M = p.M;
    r.N = p.N;
    r.C = p.C;
    r.ldc = p.ldc;
    r.sC = p.sC;
    r.ws = p.ws;
    splitk_reduce(r, batch, S, st);
    return;
  }
  const long long n = (long long)batch * p.M * (p.N / 4);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (epi == EPI_BIAS_RELU)
    hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_BIAS_RELU>, grid, dim3(256), 0, st, p, S, batch);
  else if (epi == EPI_RELU_MASK)
    hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_RELU_MASK>, grid, dim3(256), 0, st, p, S, batch);
  else
    hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_STORE>, grid, dim3(256), 0, st, p, S, batch);
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
  // ~256 rows per chunk keeps every lane streaming; COLSUM_CHUNKS bounds the partials
  const int chunks = std::max(1, std::min(COLSUM_CHUNKS, (rows + 255) / 256));
  if (cols % 4 == 0 && ld % 4 == 0 && sx % 4 == 0)
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((cols + 255) / 256, chunks, batch), dim3(256), 0, st, x, rows, cols,
                       ld, sx, chunks, part);
  else
    hipLaunchKernelGGL(colsum_partial_scalar_kernel, dim3((cols + 255) / 256, chunks, batch), dim3(256), 0, st, x,
                       rows, cols, ld, sx, chunks, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 255) / 256, 1, batch), dim3(256), 0, st, part, cols, chunks, db,
                     sdb);
}

}  // namespace mtsac
