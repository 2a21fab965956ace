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

#include "gemm_x3f_impl.h"

namespace mtsac {
namespace x3fk {

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
// tile order inside an XCD's run (experiments; SplitGemmParams::order): row tiles fastest measured
// 2.5 % slower at S3 split2h than column tiles fastest (profiles/r4h_*)
static const int g_x3f_order = [] {
  const char* e = getenv("MTSAC_X3F_ORDER");
  return e ? atoi(e) : 0;
}();

template <int EPI, bool C_OUT, bool P_OUT, bool MASK16, int TAG = 0>
void launch(const SplitGemmParams& p0, dim3 grid, hipStream_t st, int bm) {
  const dim3 blk(512);
  SplitGemmParams p = p0;
  if (g_x3f_order) p.order = g_x3f_order;
  if (p.np == 2) {  // split2h: two fp16 planes, 3 products
    hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI, C_OUT, P_OUT, MASK16, TAG, 2>), grid, blk, 0, st, p);
    return;
  }
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
    case 128: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 128, NP, WV>), grid, blk, 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 0, NP, WV>), grid, blk, 0, st, p); break;
  }
}
}  // namespace x3fk

// experiments: the bench-shape forward (bias+ReLU, planes out) with ablation bits abl (+ 1000: the
// 4-wave, 64-column-slab workgroup); precision bf16 runs the 400-row tile
void gemm_x3f_ablate(const SplitGemmParams& p, int abl, int batch, hipStream_t st) {
  using namespace x3fk;
  const bool wv4 = abl >= 1000 && abl < 2000, short8 = abl >= 2000 && abl < 3000, c2 = abl >= 3000;
  abl %= 1000;
  // bf16: + 1000 / + 2000 = 208 rows, 4 / 8 waves; + 3000 = the 80-row tile of MT10's 1280 rows (C2)
  const int bm = c2 ? 80 : p.np == 1 && !wv4 && !short8 ? 400 : BM0;
  const dim3 grid((unsigned)(((p.M + bm - 1) / bm) * ((p.N + BN - 1) / BN) * batch));
  if (p.np == 1) {
    if (c2) ablate_at<80, 1, 8>(p, abl, grid, st);
    else if (wv4) ablate_at<BM0, 1, 4>(p, abl, grid, st);
    else if (short8) ablate_at<BM0, 1, 8>(p, abl, grid, st);
    else ablate_at<400, 1, 8>(p, abl, grid, st);
  } else if (p.np == 2) {  // split2h: 8 waves, or (+ 1000) 4 waves x 64-column slabs
    if (wv4) ablate_at<BM0, 2, 4>(p, abl, grid, st);
    else ablate_at<BM0, 2, 8>(p, abl, grid, st);
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
int splitk_dbp_rows();
int gemm_x3f_max_row_tiles(int M) { return (M + splitk_dbp_rows() - 1) / splitk_dbp_rows(); }  // finest dbp chunking

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

static int x3f_slices(const SplitGemmParams& p, int epi, int batch);
int splitk_dbp_rows();
static bool x3f_fin_ok(const SplitGemmParams& p, int epi, int batch);
int gemm_x3f_out_bm(const SplitGemmParams& p, int epi, int batch) {
  if (x3f_slices(p, epi, batch) <= 1) return gemm_x3f_bm(p, batch);
  // split: the in-launch finish keeps the row tile; the finishing pass sums FR-row chunks
  return x3f_fin_ok(p, epi, batch) ? x3fk::split_plan(p.M, p.N, p.K, batch).bm : splitk_dbp_rows();
}
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
bool gemm_x3f_fin_supported(const SplitGemmParams& q, int epi, int bm);
bool gemm_x3f_fin(const SplitGemmParams& q, int epi, int bm, dim3 grid, hipStream_t st);

// the in-launch finish applies to this split launch (counters given, an instance for its outputs,
// the tiles within the counter array)
static bool x3f_fin_ok(const SplitGemmParams& p, int epi, int batch) {
  if (p.cnt == nullptr) return false;
  const x3fk::SplitPlan sp = x3fk::split_plan(p.M, p.N, p.K, batch);
  if (p.np == 2 && sp.s != 2) return false;  // split2h: the two-slice pair hand-off only
  const long long tiles = (long long)((p.M + sp.bm - 1) / sp.bm) * ((p.N + x3fk::BN - 1) / x3fk::BN) * batch;
  return tiles <= GEMM_X3F_CNT && gemm_x3f_fin_supported(p, epi, sp.bm);
}

static int x3f_slices(const SplitGemmParams& p, int epi, int batch) {
  if (p.splits >= 0 || p.ws == nullptr) return 1;
  // column sums (dbp): the in-launch finish, or the finishing pass by FR-row chunks (mask16 / bias)
  if (p.dbp != nullptr && !x3f_fin_ok(p, epi, batch) && !(epi == EPI_BIAS_RELU || (epi == EPI_RELU_MASK && p.mask16)))
    return 1;
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
         (p.C || p.Cp) && (long long)p.N * p.ldb * 2 < (1ll << 31) &&
         (!p.b_frag || (p.N % 16 == 0 && p.ldb % 32 == 0));
}

int gemm_x3f(const SplitGemmParams& p0, int epi, int batch, hipStream_t st) {
  using namespace x3fk;
  const int S = x3f_slices(p0, epi, batch);
  if (S > 1 && x3f_fin_ok(p0, epi, batch)) {  // one launch: slabs, tickets, the last slice finishes
    SplitGemmParams q = p0;
    q.kchunk = (p0.K / KS + S - 1) / S * KS;
    q.splits = (p0.K + q.kchunk - 1) / q.kchunk;
    const int bm = split_plan(p0.M, p0.N, p0.K, batch).bm;
    const unsigned tiles = (unsigned)(((p0.M + bm - 1) / bm) * ((p0.N + BN - 1) / BN) * batch);
    const dim3 grid(tiles * (unsigned)q.splits);
    if (q.splits > 1 && (q.np != 2 || q.splits == 2) && gemm_x3f_fin(q, epi, bm, grid, st)) {
      if (p0.nparts) *p0.nparts = (int)tiles;  // split2h: one partial max per tile (at the tile's index)
      return q.splits;
    }
  }
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
    switch (bm * 4 + (p0.np == 1 ? 1 : p0.np == 2 ? 2 : 3)) {
      case BMS * 4 + 2: hipLaunchKernelGGL((gemm_x3f_kernel<BMS, EPI_STORE, true, false, false, 0, 2>), grid, blk, 0, st, q); break;
      case BM0 * 4 + 2: hipLaunchKernelGGL((gemm_x3f_kernel<BM0, EPI_STORE, true, false, false, 0, 2>), grid, blk, 0, st, q); break;
      case BMT * 4 + 2: hipLaunchKernelGGL((gemm_x3f_kernel<BMT, EPI_STORE, true, false, false, 0, 2>), grid, blk, 0, st, q); break;
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
  if (p.nparts) *p.nparts = (int)grid.x;
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
