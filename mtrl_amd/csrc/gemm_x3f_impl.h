// gemm_x3f_impl.h -- the gemm_x3f kernel template (see gemm_x3f.hip for the design notes); included
// by gemm_x3f.hip (plain and raw-slab split-K instances) and gemm_x3f_fin.hip (split-K with the
// in-launch finish).
#pragma once
#include <type_traits>

#include "gemm_x3p_impl.h"

#ifndef X3F_DEEP_B
#define X3F_DEEP_B 1  // the bf16 instances' four-buffer B ring (DEEP below); 0: build without (A/B)
#endif
#ifndef X3F_EPI_GROUP
#define X3F_EPI_GROUP 2  // 16-row blocks per epilogue barrier in the plane kernels (4 measured equal: profiles/r4k_*)
#endif

namespace mtsac {
namespace x3fk {

using x3pk::glds16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BN = 256;  // 8 waves x 32 columns
constexpr int TAG_INPUT = 8;
constexpr int KS = 64;   // k per stage / main-loop step

// One B fragment: 16 B of row n at byte offset voff from the wave-uniform base (no compiler wait)
__device__ inline bf16x8 gload_frag(const __bf16* base, unsigned voff) {
  bf16x8 r;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(voff), "s"(base) : "memory");
  return r;
}

// s_waitcnt vmcnt(N) that also pins the B fragments it covers (the compiler cannot see the asm loads)
template <int N, int NP, int JB>
__device__ inline void wait_vm(bf16x8 (&b)[JB][NP]) {
  if constexpr (JB == 2 && NP == 3)
    asm volatile("s_waitcnt vmcnt(%6)"
                 : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[0][2]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[1][2])
                 : "n"(N)
                 : "memory");
  else if constexpr (JB == 2 && NP == 2)
    asm volatile("s_waitcnt vmcnt(%4)"
                 : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1])
                 : "n"(N)
                 : "memory");
  else if constexpr (NP == 2)
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[2][0]), "+v"(b[2][1]),
                   "+v"(b[3][0]), "+v"(b[3][1])
                 : "n"(N)
                 : "memory");
  else if constexpr (JB == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(b[0][0]), "+v"(b[1][0]) : "n"(N) : "memory");
  else if constexpr (NP == 3)
    asm volatile("s_waitcnt vmcnt(%12)"
                 : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[0][2]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[1][2]),
                   "+v"(b[2][0]), "+v"(b[2][1]), "+v"(b[2][2]), "+v"(b[3][0]), "+v"(b[3][1]), "+v"(b[3][2])
                 : "n"(N)
                 : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(b[0][0]), "+v"(b[1][0]), "+v"(b[2][0]), "+v"(b[3][0]) : "n"(N) : "memory");
}

// ABL: ablation bits for experiments only (tools/x3f_ablate.py; results are wrong): 1 = no A
// refills after the prologue, 2 = no B reloads after the prologue, 4 = s_setprio 1 for waves 4-7,
// 64 = each B wave-instruction reads 1 KB contiguous (8 full lines) instead of 16 rows x 64 B,
// 128 = no epilogue stores (131: no loads or stores -- MFMA, LDS reads and barriers only; interleaving
// two row tiles' MFMA chains changed nothing there).
// ABL == TAG_INPUT changes nothing: it only gives input-layer launches their own kernel symbol, so
// rocprof stats and PMC passes separate them from the hidden layers.
// NP: operand planes read (3: 6 products, fp32-accurate; 1: the high plane only, precision bf16;
// 2: precision split2h -- two fp16 planes of x 2^e per operand, 3 products h*l, l*h, h*h, the
// accumulator unscaled by 2^-(eA + eB) in the epilogue, output planes at the exponent of the bound)
// WV: waves per workgroup.  8 (two per SIMD): wave w owns the BM x 32 column slab [32w, 32w + 32);
// 4 (one per SIMD, up to 512 registers): BM x 64 slabs, so each A fragment read from LDS feeds twice
// the MFMAs (4 column fragments) -- half the LDS traffic per product, the bound of the one-plane
// (bf16) kernel, whose 8-wave skeleton saturates the LDS (256 B/clk/CU at the MFMA rate).
// FIN (split-K with the in-launch finish, p.splits > 1, p.cnt): every slice writes its raw partial
// slab to p.ws ([z][S][M][N]) and draws a ticket from the tile's arrival counter (plain stores, one
// agent-scope release, relaxed agent-scope fetch_add: cdna_hip_programming.md, 'In-launch split-K
// reduction'); the slice that draws S - 1 acquires, adds the slabs in slice order with its own
// partial standing in for its slab (bitwise the separate finishing pass's sums), applies the real
// epilogue (C / planes / column sums) and re-arms the counter.
template <int BM, int EPI, bool C_OUT, bool P_OUT, bool MASK16, int ABL = 0, int NP = 3, int WV = 8, bool FIN = false>
__global__ __launch_bounds__(64 * WV, 1) void gemm_x3f_kernel(SplitGemmParams p) {
  constexpr int JB = BN / 16 / WV;       // 16-column fragments per wave (2 or 4)
  constexpr int TI = BM / 16;            // 16-row accumulator tiles per wave
  constexpr int PLANE = BM * 128;        // bytes of one plane of one stage
  constexpr int STAGE = NP * PLANE;
  constexpr int NJ = NP * BM / 8;        // DMA wave-instructions per stage
  constexpr int PMAX = (NJ + WV - 1) / WV;  // per wave (the first NJ % WV waves), others PMAX - 1
  // every piece of the next stage is issued in the FIRST half step (spread over its row tiles), so
  // each has at least a half step to land before the drain at the next step's barrier
  constexpr int P0 = (ABL & 512) ? (PMAX + 1) / 2 : PMAX;  // 512: the old even split (experiments)
  constexpr int PW = (ABL & 512) ? P0 : PMAX - 1;  // pieces every wave has issued after B(kt, 1)
  // the epilogue reuses the ring as scratch: two 16 x (BN + 4) fp32 row-block images + 8 x BN
  // column-sum partials -- more than the ring of the short one-plane tiles holds
  // EG 16-row blocks per epilogue barrier: 2 for the plane kernels without the in-launch finish (the
  // per-block barrier chain, not the store bandwidth, bounds an epilogue-heavy launch such as the
  // input layer's), 1 otherwise
  constexpr int EG = (!FIN && NP >= 2) ? X3F_EPI_GROUP : 1;
  constexpr int EPI_LDS = (2 * EG * 16 * (BN + 4) + WV * BN + 16) * 4;  // + the split2h max scratch
  // DEEP (precision bf16, one plane; the non-split epilogue instances of up to 208 rows -- the 400-row
  // tile has no registers for the ring): B fragments run THREE half steps ahead through a ring of four
  // register buffers instead of one.  The one-plane step has a third of the MFMAs of a split2h step, so a
  // half step of MFMAs no longer covers an L2 / MALL load: at MT10's 80-row tile (C2) the kernel
  // without B reloads took 21.7 against 30.8 us (profiles/r5ah_x3f_c2_ablate.txt).
  // The same ring for the split2h tiles (three buffers at 208 rows, where four spill; four at <= 128)
  // and a staggered two-waves-per-SIMD schedule with a 3-stage LDS ring were built, passed parity and
  // measured no faster (commits f56d1da, 5207f51, 6f6b182), so removed.
  constexpr bool DEEP = NP == 1 && BM <= 208 && ABL == 0 && EPI != EPI_STORE && !FIN && X3F_DEEP_B;
  constexpr int SMEM0 = 2 * STAGE > EPI_LDS ? 2 * STAGE : EPI_LDS;
  constexpr int SMEM = SMEM0 + (FIN ? 16 : 0);  // FIN: the 'last slice' word after the scratch
  static_assert(BM % 16 == 0 && SMEM <= 160 * 1024, "tile");
  static_assert(PMAX - 1 >= PW || NJ % WV == 0, "every wave issues >= PW pieces in the first half step");
  static_assert(JB * 16 * WV == BN && (JB == 2 || JB == 4), "column slabs");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const unsigned lds_base = (unsigned)(unsigned long long)(x3pk::lds_void*)smem;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  __builtin_assume(wave >= 0 && wave < WV);
  const int mine = (wave < NJ % WV || NJ % WV == 0) ? PMAX : PMAX - 1;  // DMA pieces of this wave

  // XCD-contiguous tile order (as gemm_x3p): N tile fastest inside an XCD's run
  const int ny = (p.N + BN - 1) / BN, nx = (p.M + BM - 1) / BM;
  int lin = blockIdx.x;
  {
    const int n = gridDim.x, q8 = n / 8, r8 = n % 8, x = lin % 8;
    lin = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + lin / 8;
  }
  // split-K (p.splits > 1): slice s of K, raw partial slab out (EPI_STORE into p.C = workspace)
  const int nsplit = p.splits > 1 ? p.splits : 1;
  const int tiles = ny * nx * (int)(gridDim.x / nsplit / (ny * nx));
  // FIN: a tile's slices adjacent (one XCD: the last arriver reads same-XCD slabs); else slice-major
  const int sl = FIN ? lin % nsplit : lin / tiles;
  lin = FIN ? lin / nsplit : lin - sl * tiles;
  const int tile_id = lin;
  const int by = p.order ? (lin / nx) % ny : lin % ny, bx = p.order ? lin % nx : (lin / ny) % nx;
  const int z = lin / (ny * nx);
  const int m0 = bx * BM, n0 = by * BN;
  const int k0 = nsplit > 1 ? sl * p.kchunk : 0;
  const __bf16* __restrict__ A = p.A + z * p.sA + k0;
  // B planes in the fragment layout (p.b_frag, frag_off): k advances 16 elements per k (512 per 32)
  const int bks = p.b_frag ? 16 : 1;
  const __bf16* B = p.B + z * p.sB + (long long)bks * k0;
  const int nk = (nsplit > 1 ? min(p.kchunk, p.K - k0) : p.K) / KS;

  // ---- A: LDS-DMA piece j of the stage at k0 into stage buffer `st` (byte address)
  auto piece = [&](int j, int k0, unsigned st) {
    const int q = j / (BM / 8), rg = j % (BM / 8);
    int row = m0 + 8 * rg + (lane >> 3);
    const int pc = lane & 7;                       // physical 16-B chunk
    const int c = pc ^ (row & 7);                  // logical chunk it holds (8 k each)
    row = row < p.M ? row : p.M - 1;               // rows past M feed discarded outputs
    glds16(A + q * p.pA + (long long)row * p.lda + k0 + 8 * c, st + q * PLANE + rg * 1024);
  };
  auto wave_piece = [&](int qi, int k0, unsigned st) {  // this wave's qi-th piece of a stage
    const int j = wave + WV * qi;
    if (j < NJ) piece(j, k0, st);
  };
  // A fragment (row tile i, 32-k half s, plane q) from stage buffer `cur`
  auto afrag = [&](const char* cur, int i, int s, int q) {
    const int r = 16 * i + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(cur + q * PLANE + r * 128 + 16 * (c ^ (r & 7)));
  };

  // ---- B: per lane, rows n0 + 16 JB wave + 16 j + (lane & 15), k chunk (lane >> 4)
  unsigned boff[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    int n = n0 + 16 * JB * wave + 16 * j + (lane & 15);
    n = n < p.N ? n : p.N - 1;
    boff[j] = (unsigned)(((long long)n * p.ldb + 8 * (lane >> 4)) * 2);
    if (p.b_frag) {  // the fragment of columns nb .. nb + 15 at k = 0: this lane's 16 B of its 1 KB
      int nb = (n0 + 16 * JB * wave + 16 * j) >> 4;
      nb = nb < (p.N >> 4) ? nb : (p.N >> 4) - 1;  // N % 16 == 0 (gemm_x3f_ok)
      boff[j] = (unsigned)(((long long)nb * (p.ldb >> 5) * 512 + 8 * lane) * 2);
    }
    if (ABL & 64) boff[j] = (unsigned)((long long)(n0 + 16 * JB * wave + 16 * j) * p.ldb * 2 + 16 * lane);
  }
  auto bload = [&](bf16x8 (&b)[JB][NP], int k) {  // the 32-deep half step at k
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const __bf16* base = B + q * p.pB + bks * k;
#pragma unroll
      for (int j = 0; j < JB; ++j) b[j][q] = gload_frag(base, boff[j]);
    }
  };

  f32x4 acc[TI][JB];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 b0[JB][NP], b1[JB][NP];
  if ((ABL & 4) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  // prologue: stage 0 + B of the first half step
#pragma unroll
  for (int qi = 0; qi < PMAX; ++qi) wave_piece(qi, 0, lds_base);
  if constexpr (!DEEP) bload(b0, 0);

  // one 64-deep step; MORE: the next stage and B half step are loaded during it (all but the last)
  auto step = [&](int kt, auto more_c) {
    constexpr bool MORE = decltype(more_c)::value;
    // stage kt and B(kt, 0) have landed for this wave; after the barrier for every wave, and
    // every wave is done with step kt-1 (its stage buffer is refilled below)
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int kn = (kt + 1) * KS;
    const unsigned nst = lds_base + ((kt + 1) & 1) * STAGE;
    const char* cur = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8(&b)[JB][NP] = s == 0 ? b0 : b1;
      if (s == 0) {
        if (!(ABL & 2) || kt == 0) bload(b1, kt * KS + 32);  // second half of this step
      } else {
        if (ABL & 1) wait_vm<0, NP, JB>(b1);
        else wait_vm<MORE ? PW : 0, NP, JB>(b1);  // B(kt, 1) landed; the DMA pieces issued after it may not have
        if (MORE && !(ABL & 2)) bload(b0, kn);  // first half of the next step
      }
      bf16x8 a[2][NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) a[0][q] = afrag(cur, 0, s, q);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        if (i + 1 < TI) {
#pragma unroll
          for (int q = 0; q < NP; ++q) a[(i + 1) & 1][q] = afrag(cur, i + 1, s, q);
        }
        if (MORE && !(ABL & 1)) {  // this half step's DMA pieces of the next stage, spread over the row tiles
          constexpr int lo = 0;
          const int a0 = s == 0 ? lo : P0, a1 = s == 0 ? P0 : PMAX;
#pragma unroll
          for (int qi = a0 + (i * (a1 - a0)) / TI; qi < a0 + ((i + 1) * (a1 - a0)) / TI; ++qi)
            if (qi < mine) wave_piece(qi, kn, nst);
        }
        const bf16x8(&x)[NP] = a[i & 1];
#pragma unroll
        for (int j = 0; j < JB; ++j) {
          f32x4 c = acc[i][j];
          if constexpr (NP == 2) {  // fp16 planes: h*l, l*h, h*h
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, x[0]), __builtin_bit_cast(f16x8, b[j][1]), c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, x[1]), __builtin_bit_cast(f16x8, b[j][0]), c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, x[0]), __builtin_bit_cast(f16x8, b[j][0]), c, 0, 0, 0);
          } else {
            if constexpr (NP == 3) {
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], b[j][1], c, 0, 0, 0);  // m*m
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][2], c, 0, 0, 0);  // h*l
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[2], b[j][0], c, 0, 0, 0);  // l*h
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][1], c, 0, 0, 0);  // h*m
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], b[j][0], c, 0, 0, 0);  // m*h
            }
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][0], c, 0, 0, 0);  // h*h
          }
          acc[i][j] = c;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // DEEP: step kt computes half steps 2kt (buffer 2P) and 2kt + 1 (2P + 1), P = kt & 1, and loads half
  // steps 2kt + 3 and 2kt + 4 into the buffers freed by 2kt - 1 and 2kt.  Every step issues the same
  // operations -- B(2kt + 3), the pieces of stage kt + 1 (spread over the first half's row tiles),
  // B(2kt + 4) -- past the end of K at clamped addresses (a few loads nobody reads; the pieces land in
  // the buffer the last step does not read, and the epilogue drains them), so every count is a
  // constant: at the start of step kt only B(2kt + 2) may still be in flight besides what is waited
  // for (at kt = 0: B(1), B(2)), and at its middle B(2kt + 2), B(2kt + 3) and >= PW pieces.
  const int klast = (nk - 1) * KS;  // the last step's k
  auto bload_c = [&](bf16x8 (&b)[JB][NP], int k) { bload(b, k < klast + 32 ? k : klast + 32); };
  auto step_deep = [&](bf16x8 (&bq)[4][JB][NP], int kt, auto par_c, auto first_c) {
    constexpr int P = decltype(par_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr int S0 = 2 * P, S1 = 2 * P + 1, L0 = (2 * P + 3) & 3, L1 = (2 * P + 4) & 3;
    constexpr int NB = JB * NP;  // B wave-instructions per half step
    wait_vm<FIRST ? 2 * NB : NB, NP, JB>(bq[S0]);  // B(2kt) and this wave's stage-kt pieces
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int kn = min((kt + 1) * KS, klast);
    const unsigned nst = lds_base + ((kt + 1) & 1) * STAGE;
    const char* cur = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s == 0) {
        bload_c(bq[L0], kt * KS + 96);
      } else {
        wait_vm<2 * NB + PW, NP, JB>(bq[S1]);
        bload_c(bq[L1], kt * KS + 128);
      }
      bf16x8(&b)[JB][NP] = s == 0 ? bq[S0] : bq[S1];
      bf16x8 a[2][NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) a[0][q] = afrag(cur, 0, s, q);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        if (i + 1 < TI) {
#pragma unroll
          for (int q = 0; q < NP; ++q) a[(i + 1) & 1][q] = afrag(cur, i + 1, s, q);
        }
        if (s == 0) {
#pragma unroll
          for (int qi = (i * PMAX) / TI; qi < ((i + 1) * PMAX) / TI; ++qi)
            if (qi < mine) wave_piece(qi, kn, nst);
        }
        const bf16x8(&x)[NP] = a[i & 1];
#pragma unroll
        for (int j = 0; j < JB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][0], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  if constexpr (DEEP) {
    // one self-contained loop per parity of nk: no asm-loaded B register is live across the branch
    if (nk & 1) {
      bf16x8 bq[4][JB][NP];
      bload_c(bq[0], 0);
      bload_c(bq[1], 32);
      bload_c(bq[2], 64);
      step_deep(bq, 0, I0{}, BT{});
      for (int kt = 1; kt < nk; kt += 2) {
        step_deep(bq, kt, I1{}, BF{});
        step_deep(bq, kt + 1, I0{}, BF{});
      }
    } else {
      bf16x8 bq[4][JB][NP];
      bload_c(bq[0], 0);
      bload_c(bq[1], 32);
      bload_c(bq[2], 64);
      step_deep(bq, 0, I0{}, BT{});
      step_deep(bq, 1, I1{}, BF{});
      for (int kt = 2; kt < nk; kt += 2) {
        step_deep(bq, kt, I0{}, BF{});
        step_deep(bq, kt + 1, I1{}, BF{});
      }
    }
  } else {
    for (int kt = 0; kt + 1 < nk; ++kt) step(kt, std::integral_constant<bool, true>{});
    step(nk - 1, std::integral_constant<bool, false>{});
  }

  // ---------------------------------------------------------------- epilogue
  // Per 16-row block, the waves' 16 x 16 JB pieces meet in an LDS image of the block's 16 x 256
  // outputs (two buffers: one barrier per block); the row pairs (2r, 2r + 1), r = wave, wave + WV,
  // ..., are finished with lane l taking 8 columns 8 (l & 31): every fp32 row leaves as 1 KB and
  // every plane row as 512 B of contiguous 16-B lane stores (whole lines), instead of 16 rows x 64 B
  // per instruction.
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // the ring is free: scratch
  __builtin_amdgcn_sched_barrier(0);
  constexpr int TS = BN + 4;  // image row stride (floats): the 4 row groups of a write land 16 banks apart
  constexpr int RP = 8 / WV;  // row pairs per wave and block
  float* img = reinterpret_cast<float*>(smem);
  // split2h: unscale the products, and the output planes' exponent from the bound (every workgroup
  // alike); the scratch for the maxima sits past the epilogue's images and column-sum partials
  float unscale = 1.f, oscale = 1.f;
  float* mscr = img + 2 * EG * 16 * TS + WV * BN;
  if constexpr (NP == 2) unscale = exp2i(-p.ra->e) * exp2i(-p.rb->e);
  float omx = 0.f;  // this lane's max |out| (split2h planes)
  const int oc = 8 * (lane & 31);
  const int col = n0 + oc;
  const bool colok = col < p.N;  // N % 8 == 0: a lane's 8 columns are all in or all out
  const long long slab = (long long)p.M * p.N;
  const float* ws_z = FIN ? p.ws + (long long)z * nsplit * slab : nullptr;
  // FIN, two slices ("pair"): the ticket comes FIRST.  The slice drawing 0 publishes its partial
  // ALREADY multiplied by unscale = 2^-(eA + eB) (write_slab; true magnitude, not MFMA-scale) in its slab with write-through (sc1) stores, drains them, and signals by adding 2 to the
  // tile's counter; the slice drawing 1 (or 3: the partial is already published) polls the counter
  // until it reads 4, re-arms it, and finishes the tile from its own registers plus the other slab,
  // read with sc1 loads (the hand-off of MI355X_MICROARCH.md's table, row 1: no acquire needed).  One
  // slab written instead of two, and the poller waits only on a slice that is already running.
  // More slices: every slice writes its slab, draws a ticket, and the last one sums the slabs.
  const bool pair = FIN && nsplit == 2;
  auto write_slab = [&](bool scale) {  // this slice's partial into its slab (sc1 stores), drained
    const __amdgpu_buffer_rsrc_t slab_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.ws + ((long long)z * nsplit + sl) * slab), (short)0, -1, 0x00020000);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      float* tb = img + (i & 1) * 16 * TS;
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) tb[(4 * (lane >> 4) + r) * TS + 16 * JB * wave + 16 * j + (lane & 15)] = acc[i][j][r];
      __syncthreads();
#pragma unroll
      for (int rp = 0; rp < RP; ++rp) {
        const int orow = 2 * (wave + WV * rp) + (lane >> 5);
        const int row = m0 + 16 * i + orow;
        if (row >= p.M || !colok) continue;
        float4 u = *reinterpret_cast<const float4*>(tb + orow * TS + oc);
        float4 v = *reinterpret_cast<const float4*>(tb + orow * TS + oc + 4);
        if (scale) {
          u.x *= unscale; u.y *= unscale; u.z *= unscale; u.w *= unscale;
          v.x *= unscale; v.y *= unscale; v.z *= unscale; v.w *= unscale;
        }
        // write-through (sc1) stores: the slab leaves the XCD's L2, so no release fence (a
        // buffer_wbl2 behind 128 KB of dirty lines per workgroup) is needed before the signal
        const unsigned o = (unsigned)(((long long)row * p.N + col) * 4);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, u), slab_rs, (int)o, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), slab_rs, (int)o + 16, 0, 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
    __syncthreads();
  };
  if constexpr (FIN) {
    int* last = reinterpret_cast<int*>(smem + SMEM0);
    if (pair) {
      if (t == 0) *last = __hip_atomic_fetch_add(p.cnt + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int tk = *last;  // block-uniform
      if (tk == 0) {
        write_slab(NP == 2);
        if (t == 0) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_fetch_add(p.cnt + tile_id, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
      }
      if (t == 0) {
        if (tk == 1)  // the first slice has not published yet: it is running, so this ends
          while (__hip_atomic_load(p.cnt + tile_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 4)
            __builtin_amdgcn_s_sleep(2);
        __hip_atomic_store(p.cnt + tile_id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      }
      __syncthreads();
    } else {
      write_slab(NP == 2);
      if (t == 0) {
        const int tk = __hip_atomic_fetch_add(p.cnt + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int me = tk == nsplit - 1;
        if (me) __hip_atomic_store(p.cnt + tile_id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
        *last = me;
      }
      __syncthreads();
      if (*last == 0) return;  // block-uniform
      if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
  }
  if constexpr (NP == 2) {
    if (P_OUT) {  // the output planes' exponent: every finishing workgroup derives it alike
      const int ec = gemm_out_exp(p, mscr);
      oscale = exp2i(ec);
      if ((FIN ? tile_id : (int)blockIdx.x) == 0 && t == 0) p.rc->e = ec;
    }
  }
  float bias[8];
  if (EPI == EPI_BIAS_RELU && colok) {
    const float4 u = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col);
    const float4 v = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col + 4);
    bias[0] = u.x; bias[1] = u.y; bias[2] = u.z; bias[3] = u.w;
    bias[4] = v.x; bias[5] = v.y; bias[6] = v.z; bias[7] = v.w;
  }
  float* C = C_OUT ? p.C + z * p.sC + (FIN ? 0ll : (long long)sl * p.M * p.ldc) : nullptr;
  __bf16* Cp = P_OUT ? p.Cp + z * p.sCp : nullptr;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums over this lane's rows (dbp)
  // FIN, two slices (task shards): the other slice's values of the next PB row blocks this lane
  // finishes are loaded in one burst, so the slab reads overlap instead of costing one round trip
  // per row block
  constexpr int PB = !FIN ? 1 : TI < 8 ? TI : 8;
  float pre[PB][8];
  static_assert(!FIN || RP == 1, "the in-launch finish runs with 8 waves (one row pair per wave and block)");
  const bool two = pair;
  const __amdgpu_buffer_rsrc_t other_rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(ws_z + (1 - sl) * slab), (short)0, -1, 0x00020000);
  auto prefetch = [&](int i0) {  // the other slice's slab: sc1 loads (the pair hand-off)
#pragma unroll
    for (int ii = 0; ii < PB; ++ii) {
      const int row = m0 + 16 * (i0 + ii) + 2 * wave + (lane >> 5);
      if (i0 + ii < TI && row < p.M && colok) {
        const int o = (int)(((long long)row * p.N + col) * 4);
        const float4 a0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(other_rs, o, 0, 16));
        const float4 a1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(other_rs, o + 16, 0, 16));
        pre[ii][0] = a0.x; pre[ii][1] = a0.y; pre[ii][2] = a0.z; pre[ii][3] = a0.w;
        pre[ii][4] = a1.x; pre[ii][5] = a1.y; pre[ii][6] = a1.z; pre[ii][7] = a1.w;
      }
    }
  };
  if (two) prefetch(0);
  // split2h data grad (ReLU mask from the activation's fp16 planes): the mask rows a lane finishes in
  // the next group of row blocks are loaded one group ahead, so their latency hides behind this
  // group's image and stores instead of stalling each row (MPF; S3 207.0-208.4 -> 208.6-209.6 steps/s
  // on one box, profiles/r5ay_x3f_mask_prefetch_ab.txt)
  constexpr bool MPF = EPI == EPI_RELU_MASK && MASK16 && NP == 2 && !FIN;
  constexpr int MG = MPF ? EG * RP : 1;
  i16x8 mbuf[2][MG][2];
  auto mask_load = [&](int i0, int b) {
#pragma unroll
    for (int g = 0; g < EG; ++g)
#pragma unroll
      for (int rp = 0; rp < RP; ++rp) {
        int row = m0 + 16 * (i0 + g) + 2 * (wave + WV * rp) + (lane >> 5);
        row = row < p.M ? row : p.M - 1;  // (rows past M are not stored)
        const __bf16* mp = p.mask16 + z * p.sMask + (long long)row * p.ldm + (colok ? col : 0);
        mbuf[b][g * RP + rp][0] = __builtin_bit_cast(i16x8, *reinterpret_cast<const bf16x8*>(mp));
        mbuf[b][g * RP + rp][1] = __builtin_bit_cast(i16x8, *reinterpret_cast<const bf16x8*>(mp + p.pMask));
      }
  };
  if constexpr (MPF) mask_load(0, 0);
#pragma unroll
  for (int i0 = 0; i0 < TI; i0 += EG) {
    float* tb0 = img + ((i0 / EG) & 1) * EG * 16 * TS;
    if constexpr (MPF) {
      if (i0 + EG < TI) mask_load(i0 + EG, ((i0 / EG) + 1) & 1);
    }
#pragma unroll
    for (int g = 0; g < EG; ++g) {
      if (i0 + g >= TI) break;
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tb0[(16 * g + 4 * (lane >> 4) + r) * TS + 16 * JB * wave + 16 * j + (lane & 15)] = acc[i0 + g][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < EG; ++g) {
    const int i = i0 + g;
    if (i >= TI) break;
    if (two && i > 0 && i % PB == 0) prefetch(i);
    float* tb = tb0 + g * 16 * TS;
#pragma unroll
    for (int rp = 0; rp < RP; ++rp) {
    const int orow = 2 * (wave + WV * rp) + (lane >> 5);
    const float4 u = *reinterpret_cast<const float4*>(tb + orow * TS + oc);
    const float4 v = *reinterpret_cast<const float4*>(tb + orow * TS + oc + 4);
    const int row = m0 + 16 * i + orow;
    if (row >= p.M || !colok) continue;
    if ((ABL & 128) && p.M > 0) continue;  // ablation: no epilogue stores (p.M > 0 keeps the MFMAs live)
    float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    if constexpr (NP == 2) {  // FIN: scale this slice's registers by unscale, as the slab's partial already is
                              // (write_slab applied it; pair: s0 + s1 commutes)
#pragma unroll
      for (int c = 0; c < 8; ++c) e[c] *= unscale;
    }
    if (two) {  // s0 + s1 (fp32 addition commutes: the same bits whichever slice finishes)
#pragma unroll
      for (int c = 0; c < 8; ++c) e[c] = e[c] + pre[i % PB][c];
    } else if constexpr (FIN) {  // sum the slabs in slice order, this slice's own partial in its place
      float o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = e[c];
      const float* w = ws_z + (long long)row * p.N + col;
      for (int s = 0; s < nsplit; ++s) {
        float x[8];
        if (s == sl) {
#pragma unroll
          for (int c = 0; c < 8; ++c) x[c] = o[c];
        } else {
          const float4 a0 = *reinterpret_cast<const float4*>(w + s * slab);
          const float4 a1 = *reinterpret_cast<const float4*>(w + s * slab + 4);
          x[0] = a0.x; x[1] = a0.y; x[2] = a0.z; x[3] = a0.w;
          x[4] = a1.x; x[5] = a1.y; x[6] = a1.z; x[7] = a1.w;
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) e[c] = s == 0 ? x[c] : e[c] + x[c];
      }
    }
    if (EPI == EPI_BIAS_RELU) {
#pragma unroll
      for (int c = 0; c < 8; ++c) e[c] = fmaxf(e[c] + bias[c], 0.f);
    }
    if (EPI == EPI_RELU_MASK) {
      if (MPF) {  // the prefetched mask rows
        const i16x8& mh = mbuf[(i0 / EG) & 1][g * RP + rp][0];
        const i16x8& ml = mbuf[(i0 / EG) & 1][g * RP + rp][1];
#pragma unroll
        for (int c = 0; c < 8; ++c) e[c] = (mh[c] > 0 || ml[c] > 0) ? e[c] : 0.f;
      } else if (MASK16 && NP == 2) {  // fp16 planes: x > 0 <=> h > 0 or l > 0 (split2h_dev)
        const __bf16* mp = p.mask16 + z * p.sMask + (long long)row * p.ldm + col;
        const i16x8 mh = __builtin_bit_cast(i16x8, *reinterpret_cast<const bf16x8*>(mp));
        const i16x8 ml = __builtin_bit_cast(i16x8, *reinterpret_cast<const bf16x8*>(mp + p.pMask));
#pragma unroll
        for (int c = 0; c < 8; ++c) e[c] = (mh[c] > 0 || ml[c] > 0) ? e[c] : 0.f;
      } else if (MASK16) {
        const bf16x8 mk = *reinterpret_cast<const bf16x8*>(p.mask16 + z * p.sMask + (long long)row * p.ldm + col);
#pragma unroll
        for (int c = 0; c < 8; ++c) e[c] = (float)mk[c] > 0.f ? e[c] : 0.f;
      } else {
        const float* mp = p.mask + z * p.sMask + (long long)row * p.ldm + col;
        const float4 a0 = *reinterpret_cast<const float4*>(mp), a1 = *reinterpret_cast<const float4*>(mp + 4);
        const float mk[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) e[c] = mk[c] > 0.f ? e[c] : 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) csum[c] += e[c];
    if (C_OUT) {
      float* cp = C + (long long)row * p.ldc + col;
      *reinterpret_cast<float4*>(cp) = make_float4(e[0], e[1], e[2], e[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(e[4], e[5], e[6], e[7]);
    }
    if (P_OUT && NP == 2) {
      f16x8 h, l;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        _Float16 a_, b_;
        split2h_dev(e[c], oscale, a_, b_);
        h[c] = a_; l[c] = b_;
        omx = fmaxf(omx, fabsf(e[c]));
      }
      __bf16* pp = Cp + (long long)row * p.ldcp + col;
      *reinterpret_cast<f16x8*>(pp) = h;
      *reinterpret_cast<f16x8*>(pp + p.pC) = l;
    } else if (P_OUT) {
      bf16x8 h, m, l;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        __bf16 a_, b_, c_;
        split3_dev(e[c], a_, b_, c_);
        h[c] = a_; m[c] = b_; l[c] = c_;
      }
      __bf16* pp = Cp + (long long)row * p.ldcp + col;
      *reinterpret_cast<bf16x8*>(pp) = h;
      if (NP == 3) {  // precision bf16 reads the high plane only
        *reinterpret_cast<bf16x8*>(pp + p.pC) = m;
        *reinterpret_cast<bf16x8*>(pp + 2 * p.pC) = l;
      }
    }
    }  // row pairs
    }  // row blocks of the group
  }
  if constexpr (NP == 2 && P_OUT) {  // this workgroup's max |out|: the next producer's bound input
    const float m = block_max_val(omx, mscr);  // (FIN: one per tile, at the tile's index)
    const int slot = FIN ? tile_id : (int)blockIdx.x;
    if (t == 0 && slot < PLANE_REC_PARTS) p.rc->amax[slot] = m;
  }
  if (p.dbp) {  // the tile's column sums: lanes l, l + 32 of every wave hold the same 8 columns
    float* red = img + 2 * EG * 16 * TS;  // [WV waves][256]
#pragma unroll
    for (int c = 0; c < 8; ++c) csum[c] += __shfl_xor(csum[c], 32);
    if (lane < 32) {
#pragma unroll
      for (int c = 0; c < 8; ++c) red[wave * BN + oc + c] = csum[c];
    }
    __syncthreads();
    if (wave == 0 && lane < 32 && colok) {
      float t[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float a = red[oc + c];
#pragma unroll
        for (int w = 1; w < WV; ++w) a += red[w * BN + oc + c];
        t[c] = a;
      }
      float* d = p.dbp + ((long long)z * nx + bx) * p.N + col;
      *reinterpret_cast<float4*>(d) = make_float4(t[0], t[1], t[2], t[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(t[4], t[5], t[6], t[7]);
    }
  }
}

}  // namespace x3fk
}  // namespace mtsac
