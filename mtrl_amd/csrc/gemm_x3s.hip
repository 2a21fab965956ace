// gemm_x3s.hip -- fp32-accurate plane GEMM for SMALL row counts (task shards, MT10): the trunk
// forward and data-grad products when gemm_x3f's 208 x 256 tiles cannot fill the chip (gfx950).
//
//   C[z][m][n] = sum_k A(m, k) B(n, k), both operands ROW-MAJOR bf16 planes ([3][rows][ld], k
//   contiguous, x = x_h + x_m + x_l exactly), K a multiple of 32 (zero padded).
//
// Why a second kernel: a rank of the 8-way MT50 job holds 6-7 tasks, B = 768-896 rows; MT10 has
// B = 1280.  With W = 2048 the output is only 896 x 2048 per ensemble member, 7168 outputs per CU.
// The per-CU tile that covers that with the least operand ingest is about 112 x 64 (ingest per
// CU ~ (BM + BN) K 6 B, MFMA work ~ BM BN K), so:
//   * one 256-thread workgroup (4 waves, one per SIMD) per 16 TI x 64 output tile, TI in 4..8
//     picked per shape so the grid is whole rounds of 256 workgroups (gemm_x3s_ti);
//   * the 4 waves split K (intra-workgroup split-K: two K ranges, even / odd 32-deep steps of a
//     range to the two waves of a pair, so they request both halves of each 128-B line
//     together): every wave owns the whole tile (TI x 4 accumulators of 16 x 16), so each
//     32-deep step loads 3 TI + 12 fragments for 24 TI MFMAs, and nothing is staged through LDS
//     or shared between waves in the main loop -- no barriers, no LDS-DMA issue cost (direct
//     buffer loads -> MFMA fragments, reloaded half a step ahead);
//   * v_mfma_f32_16x16x32_bf16, 6 products per tile and 32-deep slice (m*m, h*l, l*h, h*m,
//     m*h, h*h: small terms first), fp32 accumulation -- the split3 arithmetic of gemm_x3f;
//   * XCD-aware order: the blocks sharing an XCD (b, b + 8, ...) take consecutive tiles with the
//     row tile fastest, so an XCD holds a few B column slabs in its L2 while A streams;
//   * epilogue: the 4 partial tiles meet in LDS (fixed order w = 0..3: deterministic), then each
//     thread finishes 4 consecutive columns of a row: bias+ReLU or ReLU mask (from the bf16
//     high plane of the activation: h > 0 <=> h_hi > 0), fp32 C (16 B per lane) and / or the
//     three bf16 planes of C (8 B per lane per plane); with p.dbp, the tile's column sums
//     (dbp[z][row tile][N], the data grad's bias-grad partials, as gemm_x3f writes them).
#include <algorithm>
#include <type_traits>

#include "gemm_x3p_impl.h"

namespace mtsac {
namespace x3sk {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BN = 64;  // 4 column blocks of 16
constexpr int NW = 4;   // waves per workgroup
constexpr int JB = 4;   // 16-column blocks per wave (all of the tile's)
constexpr int TAG_INPUT = 8;
// experiments only (results wrong, tools/x3s_ablate.py): TAG bit 16 = no operand loads after the
// prologue, bit 32 = no MFMAs
constexpr int ABL_NOLOAD = 16, ABL_NOMFMA = 32;

// NP: operand planes read (3: 6 products, fp32-accurate; 1: the high plane only, precision bf16;
// 2: precision split2h, two fp16 planes of x 2^e, 3 products, unscaled in the epilogue)
template <int TI, int EPI, bool C_OUT, bool P_OUT, bool MASK16, int TAG = 0, int NP = 3>
__global__ __launch_bounds__(256, 1) void gemm_x3s_kernel(SplitGemmParams p) {
  constexpr int BM = 16 * TI;
  constexpr int RLD = BN + 4;  // floats per row of a wave's partial tile in LDS
  __shared__ __attribute__((aligned(16))) float red[NW * BM * RLD];
  __shared__ float mscr[16];  // split2h: block reductions of maxima

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);

  // XCD-contiguous tile order (blocks b, b + 8, ... share an XCD), row tile fastest
  const int nx = (p.M + BM - 1) / BM, ny = (p.N + BN - 1) / BN;
  int lin = blockIdx.x;
  {
    const int n = gridDim.x, q8 = n / 8, r8 = n % 8, x = lin % 8;
    lin = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + lin / 8;
  }
  const int bx = lin % nx, by = (lin / nx) % ny, z = lin / (nx * ny);
  const int m0 = bx * BM, n0 = by * BN;
  const __bf16* __restrict__ A = p.A + z * p.sA;
  const __bf16* __restrict__ B = p.B + z * p.sB;

  // This wave's 32-deep K steps.  K is cut into two ranges at a 64-deep boundary; waves 2r and
  // 2r + 1 share range r and take its even / odd steps, so the two halves of every 128-B operand
  // line are requested by two waves of the CU at about the same time (the second one an L1 hit)
  // rather than one wave a step apart (by then evicted: every row is then fetched from L2 twice).
  const int nsteps = p.K / 32, half = ((nsteps + 3) / 4) * 2;
  const int s0 = (wave >> 1) ? half : 0, s1 = (wave >> 1) ? nsteps : min(half, nsteps);
  const int first = s0 + (wave & 1);
  const int cnt = s1 > first ? (s1 - first + 1) / 2 : 0;  // steps first, first + 2, ...
  auto kstep = [&](int u) { return 32 * (first + 2 * u); };

  // fragment addresses (elements): lane holds row (lane & 15), k chunk 8 (lane >> 4)
  const int kof = 8 * (lane >> 4);
  unsigned aoff[TI], boff[JB];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int r = min(m0 + 16 * i + (lane & 15), p.M - 1);  // rows past M feed discarded outputs
    aoff[i] = (unsigned)(2 * (r * p.lda + kof));  // bytes
  }
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int n = min(n0 + 16 * j + (lane & 15), p.N - 1);
    boff[j] = (unsigned)(2 * (n * p.ldb + kof));
  }
  // operand loads: buffer loads with a per-lane 32-bit byte offset (row / column, k chunk) and a
  // wave-uniform scalar offset (plane, k), so addressing costs TI + 4 VGPRs in all and the compiler
  // still tracks every load's vmcnt
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, -1, 0x00020000);
  auto load_a = [&](bf16x8 (&a)[NP], int i, int k) {
#pragma unroll
    for (int q = 0; q < NP; ++q)
      a[q] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff[i], (int)(2 * (q * p.pA + k)), 0));
  };
  auto load_bh = [&](bf16x8 (&b)[JB][NP], int j0, int k) {  // column blocks j0 .. j0 + JB / 2 - 1
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
      for (int j = j0; j < j0 + JB / 2; ++j)
        b[j][q] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, boff[j], (int)(2 * (q * p.pB + k)), 0));
  };

  f32x4 acc[TI][JB];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Registers: every fragment single-buffered, reloaded for the next 32-deep step right after its
  // last use in this one.  A step runs in two halves over the wave's column blocks (first half,
  // second half), all row blocks each: the first half's B blocks reload during the second half,
  // the second half's B blocks and A row block i (after its second-half MFMAs) half a step or more
  // ahead of their next use.  Every step body is straight-line code (MORE is a template
  // constant), with scheduling barriers between its groups.
  bf16x8 a[TI][NP], b[JB][NP];
  // One 16 x 16 output block, 32-deep slice: the 6 split products accumulated IN PLACE.  Inline asm
  // with the accumulator tied ("+a"): with the builtin the compiler rotates the accumulators of
  // this loop through a scratch AGPR quad (4 moves + an MFMA drain per chain).  Hazards the
  // compiler no longer sees: back-to-back MFMAs on the same exactly-overlapped accumulator need no
  // wait states; the epilogue drains the pipe (s_nop) before it reads the accumulators.
  auto mfma6 = [&](int i, int j) {
    if (TAG & ABL_NOMFMA) return;
    if constexpr (NP == 1) {
      asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[i][0]), "v"(b[j][0]));  // h*h
      return;
    }
    if constexpr (NP == 2) {  // fp16 planes: h*l, l*h, h*h
      asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %3, %4, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
          : "+a"(acc[i][j])
          : "v"(a[i][0]), "v"(b[j][1]), "v"(a[i][1]), "v"(b[j][0]));
      return;
    }
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"   // m*m
        "v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\t"   // h*l
        "v_mfma_f32_16x16x32_bf16 %0, %5, %6, %0\n\t"   // l*h
        "v_mfma_f32_16x16x32_bf16 %0, %3, %2, %0\n\t"   // h*m
        "v_mfma_f32_16x16x32_bf16 %0, %1, %6, %0\n\t"   // m*h
        "v_mfma_f32_16x16x32_bf16 %0, %3, %6, %0"         // h*h
        : "+a"(acc[i][j])
        : "v"(a[i][1]), "v"(b[j][1]), "v"(a[i][0]), "v"(b[j][2]), "v"(a[i][2]), "v"(b[j][0]));
  };
  auto step = [&](int next, auto more_c) {
    constexpr bool MORE = decltype(more_c)::value && !(TAG & ABL_NOLOAD);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int j = 0; j < JB / 2; ++j) mfma6(i, j);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (MORE) load_bh(b, 0, next);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int j = JB / 2; j < JB; ++j) mfma6(i, j);
      __builtin_amdgcn_sched_barrier(0);
      if (MORE) load_a(a[i], i, next);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (MORE) load_bh(b, JB / 2, next);
    __builtin_amdgcn_sched_barrier(0);
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  // Two steps per loop iteration (a single-step body makes the compiler rotate the accumulator
  // registers through a scratch quad, one dependent chain at a time); an odd step count gets a
  // leading phantom step on zero A fragments (it adds nothing), so the loop is pairs of steps
  // followed by one closing pair: a single control path.
  if (cnt > 0) {
    int u = 0;
    if (cnt & 1) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int q = 0; q < NP; ++q) a[i][q] = bf16x8{};
      u = -1;  // the phantom step loads step 0 as its next
    } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) load_a(a[i], i, kstep(0));
    }
    load_bh(b, 0, kstep(0));
    load_bh(b, JB / 2, kstep(0));
    for (; u + 2 < cnt; u += 2) {
      step(kstep(u + 1), T_{});
      step(kstep(u + 2), T_{});
    }
    step(kstep(u + 1), T_{});
    step(0, F_{});
  }

  // ---------------------------------------------------------------- epilogue
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA results -> reads (see mfma6)
  // partial tile of this wave -> red[wave][row][col]; accumulator element r of block (i, j) is
  // row 16 i + 4 (lane >> 4) + r, column 16 j + (lane & 15)
  {
    float* my = red + wave * (BM * RLD);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) my[(16 * i + 4 * (lane >> 4) + r) * RLD + 16 * j + (lane & 15)] = acc[i][j][r];
  }
  __syncthreads();
  // each thread finishes 4 consecutive columns of a row: 16 threads per 64-column row
  const int c4 = 4 * (t & 15);
  const int col = n0 + c4;
  const bool colok = col < p.N;  // N % 4 == 0: a thread's 4 columns are all in or all out
  const float* part = red + c4;
  float bias[4] = {0.f, 0.f, 0.f, 0.f};
  if (EPI == EPI_BIAS_RELU && colok) {
    const float4 u = *reinterpret_cast<const float4*>(p.bias + z * p.sBias + col);
    bias[0] = u.x; bias[1] = u.y; bias[2] = u.z; bias[3] = u.w;
  }
  float csum[4] = {0.f, 0.f, 0.f, 0.f};  // column sums over this thread's rows (dbp)
  float unscale = 1.f, oscale = 1.f, omx = 0.f;
  if constexpr (NP == 2) {
    unscale = exp2i(-p.ra->e) * exp2i(-p.rb->e);
    if (P_OUT) {
      const int ec = gemm_out_exp(p, mscr);
      oscale = exp2i(ec);
      if (blockIdx.x == 0 && t == 0) p.rc->e = ec;
    }
  }
  for (int rr = t >> 4; rr < BM; rr += NW * 4) {  // row in the tile
    const int row = m0 + rr;
    if (row >= p.M || !colok) break;
    float e[4];
    {  // the four partials in a fixed order: deterministic
      const float4 v0 = *reinterpret_cast<const float4*>(part + 0 * BM * RLD + rr * RLD);
      const float4 v1 = *reinterpret_cast<const float4*>(part + 1 * BM * RLD + rr * RLD);
      const float4 v2 = *reinterpret_cast<const float4*>(part + 2 * BM * RLD + rr * RLD);
      const float4 v3 = *reinterpret_cast<const float4*>(part + 3 * BM * RLD + rr * RLD);
      e[0] = ((v0.x + v1.x) + v2.x) + v3.x;
      e[1] = ((v0.y + v1.y) + v2.y) + v3.y;
      e[2] = ((v0.z + v1.z) + v2.z) + v3.z;
      e[3] = ((v0.w + v1.w) + v2.w) + v3.w;
    }
    if constexpr (NP == 2) {
#pragma unroll
      for (int c = 0; c < 4; ++c) e[c] *= unscale;
    }
    if (EPI == EPI_BIAS_RELU) {
#pragma unroll
      for (int c = 0; c < 4; ++c) e[c] = fmaxf(e[c] + bias[c], 0.f);
    }
    if (EPI == EPI_RELU_MASK) {
      static_assert(MASK16 || EPI != EPI_RELU_MASK, "ReLU mask from the bf16 high plane only");
      const __bf16* mp = p.mask16 + z * p.sMask + (long long)row * p.ldm + col;
      if constexpr (NP == 2) {  // fp16 planes: x > 0 <=> h > 0 or l > 0
        const i16x4 mh = __builtin_bit_cast(i16x4, *reinterpret_cast<const bf16x4*>(mp));
        const i16x4 ml = __builtin_bit_cast(i16x4, *reinterpret_cast<const bf16x4*>(mp + p.pMask));
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = (mh[c] > 0 || ml[c] > 0) ? e[c] : 0.f;
      } else {
        const bf16x4 mk = *reinterpret_cast<const bf16x4*>(mp);
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = (float)mk[c] > 0.f ? e[c] : 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) csum[c] += e[c];
    if (C_OUT)
      *reinterpret_cast<float4*>(p.C + z * p.sC + (long long)row * p.ldc + col) = make_float4(e[0], e[1], e[2], e[3]);
    if (P_OUT && NP == 2) {
      f16x4 h, l;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        _Float16 a_, b_;
        split2h_dev(e[c], oscale, a_, b_);
        h[c] = a_; l[c] = b_;
        omx = fmaxf(omx, fabsf(e[c]));
      }
      __bf16* pp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
      *reinterpret_cast<f16x4*>(pp) = h;
      *reinterpret_cast<f16x4*>(pp + p.pC) = l;
    } else if (P_OUT) {
      bf16x4 h, m, l;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        __bf16 a_, b_, c_;
        split3_dev(e[c], a_, b_, c_);
        h[c] = a_; m[c] = b_; l[c] = c_;
      }
      __bf16* pp = p.Cp + z * p.sCp + (long long)row * p.ldcp + col;
      *reinterpret_cast<bf16x4*>(pp) = h;
      *reinterpret_cast<bf16x4*>(pp + p.pC) = m;
      *reinterpret_cast<bf16x4*>(pp + 2 * p.pC) = l;
    }
  }
  if constexpr (NP == 2 && P_OUT) {  // this workgroup's max |out|: the next producer's bound input
    const float m = block_max_val(omx, mscr);
    if (t == 0 && blockIdx.x < PLANE_REC_PARTS) p.rc->amax[blockIdx.x] = m;
  }
  if (p.dbp) {  // the tile's column sums (the next weight grad's bias grad, finished by colsum_finish):
    // the 16 row groups (t >> 4) added in order
    __syncthreads();  // every partial-tile read is done: red is scratch
    *reinterpret_cast<float4*>(red + (t >> 4) * BN + c4) = make_float4(csum[0], csum[1], csum[2], csum[3]);
    __syncthreads();
    if (t < 16 && colok) {
      float4 a = *reinterpret_cast<const float4*>(red + c4);
      for (int g = 1; g < 16; ++g) {
        const float4 b = *reinterpret_cast<const float4*>(red + g * BN + c4);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      *reinterpret_cast<float4*>(p.dbp + ((long long)z * nx + bx) * p.N + col) = a;
    }
  }
}

template <int TI, int EPI, bool C_OUT, bool P_OUT, bool MASK16, int TAG = 0>
void launch(const SplitGemmParams& p, int batch, hipStream_t st) {
  const unsigned grid = (unsigned)(((p.M + 16 * TI - 1) / (16 * TI)) * ((p.N + BN - 1) / BN) * batch);
  if (p.nparts) *p.nparts = (int)grid;
  if (p.np == 1)
    hipLaunchKernelGGL((gemm_x3s_kernel<TI, EPI, C_OUT, P_OUT, MASK16, TAG, 1>), dim3(grid), dim3(64 * NW), 0, st, p);
  else if (p.np == 2)
    hipLaunchKernelGGL((gemm_x3s_kernel<TI, EPI, C_OUT, P_OUT, MASK16, TAG, 2>), dim3(grid), dim3(64 * NW), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_x3s_kernel<TI, EPI, C_OUT, P_OUT, MASK16, TAG, 3>), dim3(grid), dim3(64 * NW), 0, st, p);
}

template <int TI>
void dispatch(const SplitGemmParams& p, int epi, int batch, hipStream_t st) {
  const bool c = p.C != nullptr, pl = p.Cp != nullptr;
  if (epi == EPI_BIAS_RELU) {
    if (p.tag == 1 && pl && !c) launch<TI, EPI_BIAS_RELU, false, true, false, TAG_INPUT>(p, batch, st);
    else if (c && pl) launch<TI, EPI_BIAS_RELU, true, true, false>(p, batch, st);
    else if (c) launch<TI, EPI_BIAS_RELU, true, false, false>(p, batch, st);
    else launch<TI, EPI_BIAS_RELU, false, true, false>(p, batch, st);
  } else {  // the ReLU mask always comes from the bf16 high plane (gemm_x3s_ok)
    if (c && pl) launch<TI, EPI_RELU_MASK, true, true, true>(p, batch, st);
    else if (c) launch<TI, EPI_RELU_MASK, true, false, true>(p, batch, st);
    else launch<TI, EPI_RELU_MASK, false, true, true>(p, batch, st);
  }
}

}  // namespace x3sk

// experiments: the (M, N, batch) forward with planes out on TI = 7, ablations abl (1 no loads,
// 2 no MFMAs)
namespace x3sk {
template <int TI>
void ablate_ti(const SplitGemmParams& p, int abl, int batch, hipStream_t st) {
  if (abl == 1) launch<TI, EPI_BIAS_RELU, false, true, false, ABL_NOLOAD>(p, batch, st);
  else if (abl == 2) launch<TI, EPI_BIAS_RELU, false, true, false, ABL_NOMFMA>(p, batch, st);
  else launch<TI, EPI_BIAS_RELU, false, true, false>(p, batch, st);
}
}  // namespace x3sk

void gemm_x3s_ablate(const SplitGemmParams& p, int abl, int batch, hipStream_t st) {
  using namespace x3sk;
  // the row tile the dispatch picks for the shape (4 .. 8 x 16 rows)
  switch (gemm_x3s_ti(p.M, p.N, batch)) {
    case 4: ablate_ti<4>(p, abl, batch, st); break;
    case 5: ablate_ti<5>(p, abl, batch, st); break;
    case 6: ablate_ti<6>(p, abl, batch, st); break;
    case 8: ablate_ti<8>(p, abl, batch, st); break;
    default: ablate_ti<7>(p, abl, batch, st); break;
  }
}

// rows per tile / 16: the fewest (rounds of 256 workgroups) x (rows per tile), ties to the smaller
// tile (more workgroups to balance the last round)
int gemm_x3s_ti(int M, int N, int batch) {
  if (M <= 0) return 4;
  int best = 4;
  long long bc = -1;
  for (int ti = 4; ti <= 8; ++ti) {
    const long long tiles = (long long)((M + 16 * ti - 1) / (16 * ti)) * ((N + x3sk::BN - 1) / x3sk::BN) * batch;
    const long long cost = ((tiles + 255) / 256) * ti;
    if (bc < 0 || cost < bc) bc = cost, best = ti;
  }
  return best;
}

bool gemm_x3s_ok(const SplitGemmParams& p, int epi, int batch) {
  if (p.b_frag) return false;  // row-major B planes only
  auto fits = [](long long rows, long long ld, long long plane_stride) {  // 32-bit byte offsets
    return 2 * (rows * ld + 2 * plane_stride) < (1ll << 31);
  };
  return !p.a_kmajor && !p.b_kmajor && p.K % 32 == 0 && p.K >= 32 && p.M >= 1 && p.N % 4 == 0 && p.lda % 8 == 0 &&
         p.ldb % 8 == 0 && (!p.C || p.ldc % 4 == 0) && (!p.Cp || p.ldcp % 4 == 0) &&
         (epi != EPI_RELU_MASK || (p.mask16 && p.ldm % 4 == 0)) && epi != EPI_STORE && (p.C || p.Cp) && batch >= 1 &&
         fits(p.M, p.lda, p.pA) && fits(p.N, p.ldb, p.pB);
}

void gemm_x3s(const SplitGemmParams& p, int epi, int batch, hipStream_t st) {
  switch (gemm_x3s_ti(p.M, p.N, batch)) {
    case 4: x3sk::dispatch<4>(p, epi, batch, st); break;
    case 5: x3sk::dispatch<5>(p, epi, batch, st); break;
    case 6: x3sk::dispatch<6>(p, epi, batch, st); break;
    case 7: x3sk::dispatch<7>(p, epi, batch, st); break;
    default: x3sk::dispatch<8>(p, epi, batch, st); break;
  }
}

}  // namespace mtsac
