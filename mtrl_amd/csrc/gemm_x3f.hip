// gemm_x3f.hip -- fp32-accurate plane GEMM for the trunk forward and data-grad products (gfx950).
//
//   C[z][m][n] = sum_k A(m, k) B(n, k), both operands ROW-MAJOR bf16 planes ([3][rows][ld], k
//   contiguous, x = x_h + x_m + x_l exactly), K a multiple of 64 (zero padded).
//
// Design (MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//   * v_mfma_f32_16x16x32_bf16: the same issue cost per flop as the 32x32x16 form but it holds a
//     higher clock under load (MI355X_MICROARCH.md, DVFS item 7); 6 products per 16x16 tile and
//     32-deep k slice (m*m, h*l, l*h, h*m, m*h, h*h: small terms first), fp32 accumulation.
//   * 512 threads = 8 waves, 2 per SIMD; the workgroup tile is BM x 256, wave w owns the BM x 32
//     column slab [32w, 32w + 32) -- 13 x 2 accumulator tiles at BM = 208 (104 AGPRs).
//   * A (the activations, shared by all 8 waves) is staged through LDS by LDS-DMA in FULL 128-B
//     lines: one stage = 64 k, one DMA wave-instruction = 8 rows x 128 B of one plane, written
//     lane-linearly into a [row][8 x 16 B] image whose 16-B chunks are XOR-swizzled by row & 7 on
//     the SOURCE address, so the fragment reads (ds_read_b128, lane = row l & 15, chunk l >> 4)
//     are bank-conflict free.  Two stages (2 x 78 KB at BM = 208), one barrier per 64-deep step,
//     the refill of the next stage spread over the current step's MFMAs.
//   * B (the weights, each wave its own 32 columns: nothing to share inside the workgroup) goes
//     straight from L2 to registers as MFMA fragments (global_load_dwordx4, 16 rows x 64 B per
//     instruction), double-buffered per 32-deep half step.  Both load queues are counted by hand
//     (inline asm), so the compiler never drains the LDS-DMA early.
//   * M is cut into BM = 208-row tiles: B = 6400 rows -> 31 row tiles x 8 column tiles = 248
//     workgroups on 256 CUs (E = 1), 496 in two full rounds (E = 2).
//   * Epilogue per 16-row block through an LDS image of the workgroup's 16 x 256 outputs, so every
//     output row leaves in whole lines (1 KB fp32, 512 B per bf16 plane); bias+ReLU or ReLU mask
//     (fp32 or the bf16 high plane of the activation: h > 0 <=> h_hi > 0 for every normal h).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "gemm_x3p_impl.h"

namespace mtsac {
namespace x3fk {

using x3pk::glds16;
typedef float f32x4 __attribute__((ext_vector_type(4)));

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
// NP: operand planes read (3: 6 products, fp32-accurate; 1: the high plane only, precision bf16)
// WV: waves per workgroup.  8 (two per SIMD): wave w owns the BM x 32 column slab [32w, 32w + 32);
// 4 (one per SIMD, up to 512 registers): BM x 64 slabs, so each A fragment read from LDS feeds twice
// the MFMAs (4 column fragments) -- half the LDS traffic per product, the bound of the one-plane
// (bf16) kernel, whose 8-wave skeleton saturates the LDS (256 B/clk/CU at the MFMA rate).
template <int BM, int EPI, bool C_OUT, bool P_OUT, bool MASK16, int ABL = 0, int NP = 3, int WV = 8>
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
  constexpr int EPI_LDS = (2 * 16 * (BN + 4) + WV * BN) * 4;
  constexpr int SMEM = 2 * STAGE > EPI_LDS ? 2 * STAGE : EPI_LDS;
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
  const int sl = lin / tiles;
  lin -= sl * tiles;
  const int by = lin % ny, bx = (lin / ny) % nx, z = lin / (ny * nx);
  const int m0 = bx * BM, n0 = by * BN;
  const int k0 = nsplit > 1 ? sl * p.kchunk : 0;
  const __bf16* __restrict__ A = p.A + z * p.sA + k0;
  const __bf16* B = p.B + z * p.sB + k0;
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
    if (ABL & 64) boff[j] = (unsigned)((long long)(n0 + 16 * JB * wave + 16 * j) * p.ldb * 2 + 16 * lane);
  }
  auto bload = [&](bf16x8 (&b)[JB][NP], int k) {  // the 32-deep half step at k
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const __bf16* base = B + q * p.pB + k;
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
  bload(b0, 0);

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
          if constexpr (NP == 3) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], b[j][1], c, 0, 0, 0);  // m*m
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][2], c, 0, 0, 0);  // h*l
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[2], b[j][0], c, 0, 0, 0);  // l*h
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][1], c, 0, 0, 0);  // h*m
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], b[j][0], c, 0, 0, 0);  // m*h
          }
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], b[j][0], c, 0, 0, 0);  // h*h
          acc[i][j] = c;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (int kt = 0; kt + 1 < nk; ++kt) step(kt, std::integral_constant<bool, true>{});
  step(nk - 1, std::integral_constant<bool, false>{});

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
  const int oc = 8 * (lane & 31);
  const int col = n0 + oc;
  const bool colok = col < p.N;  // N % 8 == 0: a lane's 8 columns are all in or all out
  float bias[8];
  if (EPI == EPI_BIAS_RELU && colok) {
    const float4 u = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col);
    const float4 v = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col + 4);
    bias[0] = u.x; bias[1] = u.y; bias[2] = u.z; bias[3] = u.w;
    bias[4] = v.x; bias[5] = v.y; bias[6] = v.z; bias[7] = v.w;
  }
  float* C = C_OUT ? p.C + z * p.sC + (long long)sl * p.M * p.ldc : nullptr;
  __bf16* Cp = P_OUT ? p.Cp + z * p.sCp : nullptr;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums over this lane's rows (dbp)
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
    const float4 u = *reinterpret_cast<const float4*>(tb + orow * TS + oc);
    const float4 v = *reinterpret_cast<const float4*>(tb + orow * TS + oc + 4);
    const int row = m0 + 16 * i + orow;
    if (row >= p.M || !colok) continue;
    if ((ABL & 128) && p.M > 0) continue;  // ablation: no epilogue stores (p.M > 0 keeps the MFMAs live)
    float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    if (EPI == EPI_BIAS_RELU) {
#pragma unroll
      for (int c = 0; c < 8; ++c) e[c] = fmaxf(e[c] + bias[c], 0.f);
    }
    if (EPI == EPI_RELU_MASK) {
      if (MASK16) {
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
    if (P_OUT) {
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
  }
  if (p.dbp) {  // the tile's column sums: lanes l, l + 32 of every wave hold the same 8 columns
    float* red = img + 2 * 16 * TS;  // [WV waves][256]
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

constexpr int BM0 = 208;

// Precision bf16 (one plane, one MFMA per product): a workgroup's 64-deep step takes BM x 256 x 64
// multiply-adds (8 BM clocks of the CU's MFMAs) against (BM + 256) x 128 B of operands (A through
// LDS, B to registers), and one CU ingests ~28 B/clk from L2 (MI355X_MICROARCH.md gather table), so
// a step costs max(8 BM, 4.57 (BM + 256)) clocks: tall tiles run at the MFMA rate (400 rows: 26 B
// per MFMA clock), short ones at the ingest rate.  The row tile is the one whose rounds of 256
// workgroups x step cost is least -- no split-K: its fp32 partial slabs cost more HBM traffic than
// a bf16 GEMM's whole operand set.  400 rows: the S3 critic (6400 x E 2) and the merged actor
// forward (2 x 6400) in one round; 208: 6400-row single-member data grads; 80 / 48: MT10's 1280
// rows (C2) without split-K.
constexpr int BF16_BM[] = {48, 80, 208, 400};

static int bf16_bm(int M, int N, int batch) {
  const long long ny = (N + 255) / 256;
  int best = BM0;
  double best_t = 1e30;
  for (int bm : BF16_BM) {
    const long long rounds = ((M + bm - 1) / bm * ny * batch + 255) / 256;
    const double t = (double)rounds * std::max(8.0 * bm, 4.57 * (bm + 256));
    if (t < best_t - 1e-9) {
      best_t = t;
      best = bm;
    }
  }
  return best;
}

static long long bf16_workgroups(int M, int N, int batch) {
  const int bm = bf16_bm(M, N, batch);
  return (long long)((M + bm - 1) / bm) * ((N + 255) / 256) * batch;
}

// The 4-wave form (WV = 4, 64-column slabs: half the LDS fragment reads per MFMA) is kept for the
// ablations only: at the S3 shape its MFMA + LDS skeleton is 3-4 % faster, but with one wave per
// SIMD the operand loads hide worse and the full kernel is 2 % (split3, 208 rows) to 20 % (bf16,
// 208 rows vs 400) slower (profiles/r3_x3f_ablate.txt).
template <int EPI, bool C_OUT, bool P_OUT, bool MASK16, int TAG = 0>
void launch(const SplitGemmParams& p, dim3 grid, hipStream_t st, int bm) {
  const dim3 blk(512);
  if (p.np != 1) {
    hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI, C_OUT, P_OUT, MASK16, TAG, 3>), grid, blk, 0, st, p);
    return;
  }
  switch (bm) {
    case 48: hipLaunchKernelGGL((gemm_x3f_kernel<48, EPI, C_OUT, P_OUT, MASK16, TAG, 1>), grid, blk, 0, st, p); break;
    case 80: hipLaunchKernelGGL((gemm_x3f_kernel<80, EPI, C_OUT, P_OUT, MASK16, TAG, 1>), grid, blk, 0, st, p); break;
    case 400: hipLaunchKernelGGL((gemm_x3f_kernel<400, EPI, C_OUT, P_OUT, MASK16, TAG, 1>), grid, blk, 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI, C_OUT, P_OUT, MASK16, TAG, 1>), grid, blk, 0, st, p); break;
  }
}

}  // namespace x3fk

namespace x3fk {
template <int BM, int NP, int WV>
void ablate_at(const SplitGemmParams& p, int abl, dim3 grid, hipStream_t st) {
  const dim3 blk(64 * WV);
  switch (abl) {
    case 1: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 1, NP, WV>), grid, blk, 0, st, p); break;
    case 2: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 2, NP, WV>), grid, blk, 0, st, p); break;
    case 3: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 3, NP, WV>), grid, blk, 0, st, p); break;
    case 64: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 64, NP, WV>), grid, blk, 0, st, p); break;
    case 131: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 131, NP, WV>), grid, blk, 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 0, NP, WV>), grid, blk, 0, st, p); break;
  }
}
}  // namespace x3fk

// experiments: the bench-shape forward (bias+ReLU, planes out) with ablation bits abl (+ 1000: the
// 4-wave, 64-column-slab workgroup); precision bf16 runs the 400-row tile
void gemm_x3f_ablate(const SplitGemmParams& p, int abl, int batch, hipStream_t st) {
  using namespace x3fk;
  const bool wv4 = abl >= 1000 && abl < 2000, short8 = abl >= 2000;
  abl %= 1000;
  const int bm = p.np == 1 && !wv4 && !short8 ? 400 : BM0;  // bf16: + 1000 / + 2000 = 208 rows, 4 / 8 waves
  const dim3 grid((unsigned)(((p.M + bm - 1) / bm) * ((p.N + BN - 1) / BN) * batch));
  if (p.np == 1) {
    if (wv4) ablate_at<BM0, 1, 4>(p, abl, grid, st);
    else if (short8) ablate_at<BM0, 1, 8>(p, abl, grid, st);
    else ablate_at<400, 1, 8>(p, abl, grid, st);
  } else if (wv4) {
    ablate_at<BM0, 3, 4>(p, abl, grid, st);
  } else if (abl == 4 || abl == 128 || abl == 512) {
    const dim3 blk(512);
    if (abl == 4) hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI_BIAS_RELU, false, true, false, 4>), grid, blk, 0, st, p);
    if (abl == 128) hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI_BIAS_RELU, false, true, false, 128>), grid, blk, 0, st, p);
    if (abl == 512) hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI_BIAS_RELU, false, true, false, 512>), grid, blk, 0, st, p);
  } else {
    ablate_at<BM0, 3, 8>(p, abl, grid, st);
  }
}

int gemm_x3f_row_tiles(int M) { return (M + x3fk::BM0 - 1) / x3fk::BM0; }
int gemm_x3f_max_row_tiles(int M) { return (M + x3fk::BF16_BM[0] - 1) / x3fk::BF16_BM[0]; }

int gemm_x3f_bm(const SplitGemmParams& p, int batch) { return p.np == 1 ? x3fk::bf16_bm(p.M, p.N, batch) : x3fk::BM0; }

namespace x3fk {
constexpr int BMS = 128;  // the split-K row tile alternatives for task shards (96 / 84 KB of LDS)
constexpr int BMT = 112;

struct SplitPlan {
  int bm, s;
};

// Row tile and split-K slices for row counts whose 208-row tiles do not fill the chip (task shards):
// least (rounds of tiles x S workgroups) x (row-tile work relative to 208 rows / its MFMA
// efficiency) / S, plus ~4 % of a round per extra slice (its partial slab traffic and the finishing
// pass); >= 4 64-deep steps per slice.  A 128-row tile wins where 208 rows leave a mostly empty last
// tile (896 rows: 4 x 208 + 64 -> 7 x 128, 2 slices instead of 3).  MTSAC_X3F_SPLIT_BM=208|128|112
// forces the row tile (experiments; 112 rows -- 8 x 8 x 2 = 256 workgroups in 2 slices at 896 rows,
// one full round -- measured no faster than 128: 2.17 vs 2.15 ms per 7-task shard step,
// profiles/r3c_shard_steps*.txt).
static SplitPlan split_plan(int M, int N, int K, int batch) {
  if ((long long)gemm_x3f_tiles(M, N, batch) >= 192) return {BM0, 1};
  static const int forced = [] {
    const char* e = getenv("MTSAC_X3F_SPLIT_BM");
    return e ? atoi(e) : 0;
  }();
  const int smax = std::min(8, std::max(1, K / KS / 4));
  SplitPlan best{BM0, 1};
  double best_cost = 1e30;
  for (int bm : {BM0, BMS, BMT}) {
    if (forced ? bm != forced : bm == BMT) continue;  // 112 rows: experiments only (no faster than 128)
    const long long tiles = (long long)((M + bm - 1) / bm) * ((N + BN - 1) / BN) * batch;
    // shorter tiles ingest more operand bytes per MFMA: ~0.9 (128 rows), ~0.85 (112) of the rate
    const double work = bm == BM0 ? 1.0 : (double)bm / BM0 / (bm == BMS ? 0.9 : 0.85);
    for (int sp = 1; sp <= smax; ++sp) {
      const double cost = (double)((tiles * sp + 255) / 256) * work / sp + 0.04 * (sp - 1);
      if (cost < best_cost - 1e-9) {
        best_cost = cost;
        best = {bm, sp};
      }
    }
  }
  return best;
}
}  // namespace x3fk

int gemm_x3f_splits(int M, int N, int K, int batch) { return x3fk::split_plan(M, N, K, batch).s; }
int gemm_x3f_split_bm(int M, int N, int K, int batch) { return x3fk::split_plan(M, N, K, batch).bm; }

long long gemm_x3f_ws_floats(int M, int N, int K, int batch) {
  const int s = gemm_x3f_splits(M, N, K, batch);
  return s > 1 ? (long long)batch * s * M * N : 0;
}

int gemm_x3f_tiles(int M, int N, int batch) {
  return ((M + x3fk::BM0 - 1) / x3fk::BM0) * ((N + x3fk::BN - 1) / x3fk::BN) * batch;
}

// slices this launch would use: 1, or gemm_x3f_splits when the caller allows split-K
// (splits < 0, a workspace given) and the finishing pass can apply the epilogue
static int x3f_slices(const SplitGemmParams& p, int epi, int batch) {
  if (p.splits >= 0 || p.ws == nullptr || p.dbp != nullptr) return 1;
  static const bool bf16_split = [] {  // experiments: split-K for the one-plane kernel too
    const char* e = getenv("MTSAC_BF16_SPLIT");
    return e && atoi(e) != 0;
  }();
  if (p.np == 1 && !bf16_split && x3fk::bf16_workgroups(p.M, p.N, batch) >= 128) return 1;
  if (epi == EPI_RELU_MASK && !p.mask16 && !p.mask) return 1;
  if (p.N % 4 != 0 || (p.C && p.ldc % 4 != 0) || (p.Cp && p.ldcp % 4 != 0)) return 1;
  return gemm_x3f_splits(p.M, p.N, p.K, batch);
}

// workgroups of the launch (all slices)
static long long x3f_workgroups(const SplitGemmParams& p, int epi, int batch) {
  const int S = x3f_slices(p, epi, batch);
  if (S == 1) return p.np == 1 ? x3fk::bf16_workgroups(p.M, p.N, batch) : gemm_x3f_tiles(p.M, p.N, batch);
  const int bm = x3fk::split_plan(p.M, p.N, p.K, batch).bm;
  return (long long)((p.M + bm - 1) / bm) * ((p.N + x3fk::BN - 1) / x3fk::BN) * batch * S;
}

bool gemm_x3f_ok(const SplitGemmParams& p, int epi, int batch) {
  return !p.a_kmajor && !p.b_kmajor && p.K % x3fk::KS == 0 && p.N % 8 == 0 && p.lda % 8 == 0 && p.ldb % 8 == 0 &&
         (!p.C || p.ldc % 4 == 0) && (!p.Cp || p.ldcp % 8 == 0) && (epi != EPI_RELU_MASK || p.ldm % 8 == 0) &&
         (epi != EPI_STORE) && x3f_workgroups(p, epi, batch) >= 192 &&
         (p.C || p.Cp) && (long long)p.N * p.ldb * 2 < (1ll << 31);
}

int gemm_x3f(const SplitGemmParams& p0, int epi, int batch, hipStream_t st) {
  using namespace x3fk;
  const int S = x3f_slices(p0, epi, batch);
  if (S > 1) {  // raw partial slabs [z][S][M][N] into the workspace, then the epilogue pass
    SplitGemmParams q = p0;
    q.splits = S;
    q.kchunk = (p0.K / KS + S - 1) / S * KS;
    q.C = p0.ws;
    q.ldc = p0.N;
    q.sC = (long long)S * p0.M * p0.N;
    q.Cp = nullptr;
    q.dbp = nullptr;
    const int S_eff = (p0.K + q.kchunk - 1) / q.kchunk;
    q.splits = S_eff;
    const int bm = split_plan(p0.M, p0.N, p0.K, batch).bm;
    const dim3 grid((unsigned)(((p0.M + bm - 1) / bm) * ((p0.N + BN - 1) / BN) * batch * S_eff));
    const dim3 blk(512);
    switch (bm * 4 + (p0.np == 1 ? 1 : 3)) {
      case BMS * 4 + 1: hipLaunchKernelGGL((gemm_x3f_kernel<BMS, EPI_STORE, true, false, false, 0, 1>), grid, blk, 0, st, q); break;
      case BMS * 4 + 3: hipLaunchKernelGGL((gemm_x3f_kernel<BMS, EPI_STORE, true, false, false, 0, 3>), grid, blk, 0, st, q); break;
      case BMT * 4 + 1: hipLaunchKernelGGL((gemm_x3f_kernel<BMT, EPI_STORE, true, false, false, 0, 1>), grid, blk, 0, st, q); break;
      case BMT * 4 + 3: hipLaunchKernelGGL((gemm_x3f_kernel<BMT, EPI_STORE, true, false, false, 0, 3>), grid, blk, 0, st, q); break;
      case BM0 * 4 + 1: hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI_STORE, true, false, false, 0, 1>), grid, blk, 0, st, q); break;
      default: hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI_STORE, true, false, false, 0, 3>), grid, blk, 0, st, q); break;
    }
    SplitGemmParams f = p0;
    f.sC = p0.sC;
    splitk_finish(f, epi, S_eff, batch, st);
    return S_eff;
  }
  const SplitGemmParams& p = p0;
  const int bm = gemm_x3f_bm(p, batch);
  const dim3 grid((unsigned)(((p.M + bm - 1) / bm) * ((p.N + BN - 1) / BN) * batch));
  const bool c = p.C != nullptr, pl = p.Cp != nullptr, m16 = p.mask16 != nullptr;
  if (epi == EPI_BIAS_RELU && p.tag == 1 && pl && !c) {
    launch<EPI_BIAS_RELU, false, true, false, TAG_INPUT>(p, grid, st, bm);  // input layer (planes out)
  } else if (epi == EPI_BIAS_RELU) {
    if (c && pl) launch<EPI_BIAS_RELU, true, true, false>(p, grid, st, bm);
    else if (c) launch<EPI_BIAS_RELU, true, false, false>(p, grid, st, bm);
    else launch<EPI_BIAS_RELU, false, true, false>(p, grid, st, bm);
  } else {
    if (m16) {
      if (c && pl) launch<EPI_RELU_MASK, true, true, true>(p, grid, st, bm);
      else if (c) launch<EPI_RELU_MASK, true, false, true>(p, grid, st, bm);
      else launch<EPI_RELU_MASK, false, true, true>(p, grid, st, bm);
    } else {
      if (c && pl) launch<EPI_RELU_MASK, true, true, false>(p, grid, st, bm);
      else if (c) launch<EPI_RELU_MASK, true, false, false>(p, grid, st, bm);
      else launch<EPI_RELU_MASK, false, true, false>(p, grid, st, bm);
    }
  }
  return 1;
}

}  // namespace mtsac
