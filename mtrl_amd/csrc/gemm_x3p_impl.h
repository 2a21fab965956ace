// gemm_x3p_impl.h -- the plane GEMM kernel template (instantiated per geometry / operand form by
// the gemm_x3p_g*.hip units, dispatched from gemm_x3p.hip): fp32-accurate GEMM on PRE-SPLIT bf16 planes (gfx950).
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
#pragma once
#include <algorithm>

#include "gemm_common.h"

namespace mtsac {

typedef f32x16_t f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

namespace x3pk {

constexpr int BK = 32;  // K granule of the operands (split-K slices, padding); K-steps are 16 or 32

typedef __attribute__((address_space(3))) void lds_void;

// One LDS-DMA wave-instruction (16 B per lane to dst + 16 * lane).  Issued from inline asm: the
// builtin makes the compiler drain every outstanding ds_read (lgkmcnt(0)) before each DMA, which
// serialises the fragment reads against the refill spread over the MFMAs.  The ring protocol
// (counted vmcnt + one barrier per K-step) orders the DMA against the reads instead; M0 carries
// the wave-uniform LDS byte address (SALU write -> LDS-DMA read of M0 needs one wait state).  M0 is a
// reserved register (clang rejects it in a clobber list: "may not be preserved"), so this relies on the
// compiler keeping no value of its own there; tests/test_isa_m0.py checks that on the built library's
// gfx950 machine code: every M0 access is this statement's write and the LDS-DMA right after it.
__device__ inline void glds16(const void* src, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src),
               "s"(__builtin_amdgcn_readfirstlane(lds_addr))
               : "memory");
}
// One operand's image of a K-step: R rows (M or N) x KS k, NP planes (3: the fp32-accurate split;
// 1: the high plane only, precision bf16).
template <int R, bool KM, int KS, int NP = 3>
struct Oper {
  static constexpr int PLANE = R * KS * 2;  // bytes per plane
  static constexpr int BYTES = NP * PLANE;
  static constexpr int NJ = NP * PLANE / 1024;  // 1-KiB wave-instructions per stage
  static constexpr int ROWB = KM ? 2 * R : 2 * KS;
  static constexpr int RPI = 1024 / ROWB;   // image rows per wave-instruction
  static constexpr int LPR = ROWB / 16;     // lanes per image row
  static constexpr int PER_PLANE = NJ / NP;
  static_assert(!KM || LPR >= 16, "k-major swizzle needs >= 16 chunks per row");

  // physical 16-B chunk of logical chunk c in image row irow (conflict-free reads, see header)
  __device__ static inline int pchunk(int irow, int c) {
    if (KM) return c ^ (4 * (irow & 3));
    return KS == 32 ? (c ^ ((irow >> 2) & 3)) : (c ^ ((irow >> 3) & 1));
  }

  // issue wave-instructions first, first + stride, ... (< NJ) of the stage at k0
  __device__ static inline void dma(const __bf16* __restrict__ base, long long ld, long long ps, int r0, int nrows,
                                    int k0, unsigned lds, int first, int stride) {
#pragma unroll
    for (int j = first; j < NJ; j += stride) dma_one(base, ld, ps, r0, nrows, k0, lds, j);
  }

  // wave-instruction j (< NJ) of the stage at k0
  __device__ static inline void dma_one(const __bf16* __restrict__ base, long long ld, long long ps, int r0, int nrows,
                                        int k0, unsigned lds, int j) {
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

// NP: operand planes read (3: 6 products per tile and slice, fp32-accurate; 1: h*h only, bf16)
// FIN (split-K weight grads, EPI_STORE, p.cnt): every slice writes its raw slab and draws a ticket
// from the tile's arrival counter (plain stores, one agent-scope release, relaxed agent fetch_add);
// the slice drawing S - 1 acquires and adds the tile's S slabs in slice order into C (the bits of
// splitk_reduce_kernel), then re-arms the counter -- no separate reduce launch.
template <class G, bool AKM, bool BKM, int EPI, bool PLANES_OUT, int NP = 3, bool FIN = false>
__global__ __launch_bounds__(G::NTH, 1) void gemm_x3p_kernel(SplitGemmParams p) {
  using OA = Oper<G::BM, AKM, G::KS, NP>;
  using OB = Oper<G::BN, BKM, G::KS, NP>;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  // the stage's wave-instructions are dealt round robin: waves < DMA_X issue one more
  constexpr int DMA_LO = (OA::NJ + OB::NJ) / G::NW, DMA_X = (OA::NJ + OB::NJ) % G::NW;
  static_assert(G::STAGES * STAGE + (FIN ? 16 : 0) <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[G::STAGES * STAGE + (FIN ? 16 : 0)];  // FIN: + the 'last' word
  char* lds = smem;
  const unsigned lds_base = (unsigned)(unsigned long long)(lds_void*)smem;  // LDS byte address

  const int ny = (p.N + G::BN - 1) / G::BN, nx = (p.M + G::BM - 1) / G::BM;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (wave % G::WM) * (G::BM / G::WM), wn = (wave / G::WM) * (G::BN / G::WN);
  const int fb = (G::NW - (OA::NJ % G::NW) + wave) % G::NW;  // B's instructions continue the round robin
  constexpr int PIECES = DMA_LO + (DMA_X ? 1 : 0);          // per wave and stage (the last maybe empty)
  constexpr int SLOTS = (G::KS / 16) * G::TI * G::TJ;        // MFMA groups per K-step

  // XCD-aware order (lin below): the grid is 1-D and consecutive workgroups land on different
  // XCDs (round robin), so each XCD gets a contiguous run of tiles, N-tile fastest -- the
  // workgroups resident on one XCD then share a few A row-blocks and every B column-block
  // through its L2.
  f32x16 acc[G::TI][G::TJ];

  // acc = sum over the nk K-steps of the operands at A, B (already moved to the first k) for the
  // tile at (m0, n0)
  auto kloop = [&](const __bf16* __restrict__ A, const __bf16* __restrict__ B, int m0, int n0, int nk) {
    auto stage = [&](int s, int k0) {
      const unsigned st = lds_base + s * STAGE;
      OA::dma(A, p.lda, p.pA, m0, p.M, k0, st, wave, G::NW);
      OB::dma(B, p.ldb, p.pB, n0, p.N, k0, st + OA::BYTES, fb, G::NW);
    };
    // the wave's q-th wave-instruction of a stage (same dealing as stage(): global index
    // wave + q * NW, A's instructions first)
    auto piece = [&](int s, int k0, int q) {
      const unsigned st = lds_base + s * STAGE;
      const int jg = wave + q * G::NW;
      if (jg < OA::NJ)
        OA::dma_one(A, p.lda, p.pA, m0, p.M, k0, st, jg);
      else if (jg - OA::NJ < OB::NJ)
        OB::dma_one(B, p.ldb, p.pB, n0, p.N, k0, st + OA::BYTES, jg - OA::NJ);
    };
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
        bf16x8 a[G::TI][NP], b[G::TJ][NP];
#pragma unroll
        for (int i = 0; i < G::TI; ++i)
#pragma unroll
          for (int q = 0; q < NP; ++q) a[i][q] = OA::frag(cur, q, wm + 32 * i, ks, lane);
#pragma unroll
        for (int j = 0; j < G::TJ; ++j)
#pragma unroll
          for (int q = 0; q < NP; ++q) b[j][q] = OB::frag(cur + OA::BYTES, q, wn + 32 * j, ks, lane);
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
            if constexpr (NP == 2) {  // fp16 planes: h*l, l*h, h*h
              typedef _Float16 h8 __attribute__((ext_vector_type(8)));
              c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a[i][0]), __builtin_bit_cast(h8, b[j][1]), c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a[i][1]), __builtin_bit_cast(h8, b[j][0]), c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a[i][0]), __builtin_bit_cast(h8, b[j][0]), c, 0, 0, 0);
              acc[i][j] = c;
              continue;
            }
            if constexpr (NP == 3) {
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);  // m*m
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);  // h*l
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);  // l*h
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);  // h*m
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);  // m*h
            }
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);  // h*h
            acc[i][j] = c;
          }
      }
    }
  };

  // epilogue of the tile at (m0, n0) of batch entry z: raw = partial slab zz (split-K), else C
  // with the epilogue and planes
  auto epilogue = [&](int z, int zz, bool raw, int m0, int n0) {
    TileOut o{};
    if (raw) {
      o.C = p.ws + (long long)zz * p.M * p.N;
      o.ldc = p.N;
    } else {
      o.C = p.C ? p.C + z * p.sC : nullptr;
      o.ldc = p.ldc;
    }
    o.bias = (EPI == EPI_BIAS_RELU) ? p.bias + z * p.sBias : nullptr;
    o.mask = (EPI == EPI_RELU_MASK) ? p.mask + z * p.sMask : nullptr;
    o.ldm = p.ldm;
    o.Cp = (PLANES_OUT && !raw) ? p.Cp + z * p.sCp : nullptr;
    o.ldcp = p.ldcp;
    o.pC = p.pC;
    o.M = p.M;
    o.N = p.N;
    o.vec = (p.N % 4 == 0) && (o.ldc % 4 == 0) && (EPI != EPI_RELU_MASK || p.ldm % 4 == 0) &&
            (!PLANES_OUT || p.ldcp % 4 == 0);
    o.h2 = NP == 2;
    o.unscale = o.oscale = 1.f;
    __builtin_amdgcn_s_barrier();  // every wave is done with the ring: reuse it as scratch
    float* mscr = reinterpret_cast<float*>(smem) + G::NW * (32 * 36);
    if constexpr (NP == 2) {
      o.unscale = exp2i(-p.ra->e) * exp2i(-p.rb->e);
      if (o.Cp) {  // block-uniform (raw is)
        const int ec = gemm_out_exp(p, mscr);
        o.oscale = exp2i(ec);
        if (blockIdx.x == 0 && t == 0) p.rc->e = ec;
      }
    }
    float omx = 0.f;
    float* scr = reinterpret_cast<float*>(smem) + wave * (32 * 36);
#pragma unroll
    for (int i = 0; i < G::TI; ++i)
#pragma unroll
      for (int j = 0; j < G::TJ; ++j) store_tile32<EPI>(acc[i][j], scr, lane, m0 + wm + 32 * i, n0 + wn + 32 * j, o, omx);
    if constexpr (NP == 2) {
      if (o.Cp) {  // this workgroup's max |out|: the next producer's bound input
        const float m = block_max_val(omx, mscr);
        if (t == 0 && blockIdx.x < PLANE_REC_PARTS) p.rc->amax[blockIdx.x] = m;
      }
    }
  };

  // one tile (or one split-K slice of one) per workgroup, XCD-contiguous order
  int lin = blockIdx.x;
  if (!(p.dbg & 4)) {
    const int n = gridDim.x, q8 = n / 8, r8 = n % 8, x = lin % 8;
    lin = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + lin / 8;
  }
  const int S = p.splits > 1 ? p.splits : 1;
  // FIN: a tile's slices adjacent (one XCD: the last arriver reads same-XCD slabs)
  const int sp0 = FIN ? lin % S : 0;
  if (FIN) lin /= S;
  const int by = lin % ny, bx = (lin / ny) % nx;
  const int z = FIN ? lin / (ny * nx) : lin / (ny * nx) / S;
  const int sp = FIN ? sp0 : lin / (ny * nx) - z * S;
  const int zz = z * S + sp;
  const long long k0 = (long long)sp * p.kchunk;
  const int nks = (S > 1 ? min(p.kchunk, p.K - (int)k0) : p.K) / G::KS;
  const int m0 = bx * G::BM, n0 = by * G::BN;
  kloop(p.A + z * p.sA + (AKM ? k0 * p.lda : k0), p.B + z * p.sB + (BKM ? k0 * p.ldb : k0), m0, n0, nks);
  epilogue(z, zz, S > 1, m0, n0);
  if constexpr (FIN) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem + G::STAGES * STAGE);
    const int tile = lin;  // (z, bx, by)
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int tk = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int me = tk == S - 1;
      if (me) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      *last = me;
    }
    __syncthreads();
    if (*last == 0) return;  // block-uniform
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // C tile = sum of the S slabs in slice order (N, ldc multiples of 4: the host checks)
    const long long slab = (long long)p.M * p.N;
    const float* w = p.ws + (long long)z * S * slab;
    float* c = p.C + z * p.sC;
    constexpr int Q = G::BN / 4;  // float4 columns per tile row
    constexpr int U = 8;          // float4s per thread in flight
    static_assert(G::BM * Q % (G::NTH * U) == 0, "reduce tiling");
    for (int e0 = t; e0 < G::BM * Q; e0 += G::NTH * U) {
      float4 a[U];
      long long off[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * G::NTH, r = m0 + e / Q, cc = n0 + 4 * (e % Q);
        ok[u] = r < p.M && cc < p.N;
        off[u] = (long long)r * p.N + cc;
        if (ok[u]) a[u] = *reinterpret_cast<const float4*>(w + off[u]);
      }
      for (int s = 1; s < S; ++s) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (ok[u]) {
            const float4 v = *reinterpret_cast<const float4*>(w + s * slab + off[u]);
            a[u].x += v.x; a[u].y += v.y; a[u].z += v.z; a[u].w += v.w;
          }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (ok[u]) {
          const int e = e0 + u * G::NTH, r = m0 + e / Q, cc = n0 + 4 * (e % Q);
          *reinterpret_cast<float4*>(c + (long long)r * p.ldc + cc) = a[u];
        }
    }
  }
}

using GeoSmall = Geo<128, 128, 2, 2, 3, 32>;   // 4 waves, 3 x 48 KiB
using GeoWide = Geo<256, 128, 4, 2, 2, 32>;    // 8 waves, 2 x 72 KiB
using GeoWide16 = Geo<256, 128, 4, 2, 4, 16>;  // 8 waves, 4 x 36 KiB
using GeoBig16 = Geo<256, 256, 2, 4, 3, 16>;   // 8 waves of 128 x 64, 3 x 48 KiB
using GeoSmall16 = Geo<128, 128, 2, 2, 3, 16>;  // 4 waves, 3 x 24 KiB: two workgroups per CU
using GeoBig16In = Geo<256, 256, 2, 4, 3, 16, 1>;  // GeoBig16 for input-layer launches (own symbol)
// 224 x 256: 8 waves of 224 x 32 (7 x 1 MFMA tiles), 3 x 45 KiB; row-major A only (the k-major
// image swizzle needs a power-of-two row count).  B = 6400 rows cut into 29 row tiles instead of
// 25: 232 / 464 tiles on 256 CUs instead of 200 / 400, each 7/8 of the work of a 256-row tile.
using GeoTall224 = Geo<224, 256, 1, 8, 3, 16>;
using GeoTall224In = Geo<224, 256, 1, 8, 3, 16, 1>;  // input-layer launches (own symbol)

template <class G, bool AKM, bool BKM, int NP>
void launch_x3p_np(const SplitGemmParams& p, int epi, dim3 grid, hipStream_t st) {
  const bool planes = p.Cp != nullptr;
  const dim3 block(G::NTH);
  if constexpr (AKM && BKM && NP == 3 && G::STAGES * (G::BM + G::BN) * G::KS * 2 * 3 + 16 <= 160 * 1024) {
    if (epi == EPI_STORE && !planes && p.cnt != nullptr && p.splits > 1) {  // weight grads: in-launch finish
      hipLaunchKernelGGL((gemm_x3p_kernel<G, true, true, EPI_STORE, false, 3, true>), grid, block, 0, st, p);
      return;
    }
  }
  if (epi == EPI_BIAS_RELU) {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_BIAS_RELU, true, NP>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_BIAS_RELU, false, NP>), grid, block, 0, st, p);
  } else if (epi == EPI_RELU_MASK) {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_RELU_MASK, true, NP>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_RELU_MASK, false, NP>), grid, block, 0, st, p);
  } else {
    if (planes) hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_STORE, true, NP>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((gemm_x3p_kernel<G, AKM, BKM, EPI_STORE, false, NP>), grid, block, 0, st, p);
  }
}

template <class G, bool AKM, bool BKM>
void launch_x3p_v(const SplitGemmParams& p, int epi, dim3 grid, hipStream_t st) {
  if (p.np == 1) launch_x3p_np<G, AKM, BKM, 1>(p, epi, grid, st);
  else if (p.np == 2) launch_x3p_np<G, AKM, BKM, 2>(p, epi, grid, st);
  else launch_x3p_np<G, AKM, BKM, 3>(p, epi, grid, st);
}

// operand forms in MASK (bit f: f = a_kmajor | 2 b_kmajor)
template <class G, int MASK>
void launch_forms(const SplitGemmParams& p, int epi, dim3 grid, hipStream_t st) {
  const int form = (p.a_kmajor ? 1 : 0) | (p.b_kmajor ? 2 : 0);
#define X3P_FORM(F, AK, BK)                      \
  if constexpr (((MASK >> F) & 1) != 0)          \
    if (form == F) {                             \
      launch_x3p_v<G, AK, BK>(p, epi, grid, st); \
      return;                                    \
    }
  X3P_FORM(0, false, false)
  X3P_FORM(1, true, false)
  X3P_FORM(2, false, true)
  X3P_FORM(3, true, true)
#undef X3P_FORM
}

}  // namespace x3pk

// per-unit entry points (gemm_x3p_g*.hip)
#define X3P_UNIT(NAME, GEO, MASK)                                           \
  void NAME(const SplitGemmParams& p, int epi, dim3 grid, hipStream_t st) { \
    x3pk::launch_forms<x3pk::GEO, MASK>(p, epi, grid, st);                  \
  }
void x3p_unit_g0(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g1(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g2(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g3f0(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g3f1(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g3f2(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g3f3(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g4(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g3in(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g5(const SplitGemmParams&, int, dim3, hipStream_t);
void x3p_unit_g5in(const SplitGemmParams&, int, dim3, hipStream_t);

}  // namespace mtsac
