/*
 * mtsac_debug.h -- test-only entry points of libmtsac.so (not part of the drop-in
 * boundary).  They expose single device kernels so the parity tests can check a
 * kernel in isolation against the oracle / a torch fp32 reference.
 */
#ifndef MTSAC_DEBUG_H_
#define MTSAC_DEBUG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One batched fp32 MFMA GEMM with epilogue on device 0 (host pointers in/out):
 *   kind 0 NN: C = A[M][K] . B[K][N]   kind 1 NT: C = A[M][K] . B[N][K]^T
 *   kind 2 TN: C = A[K][M]^T . B[K][N]
 *   epi 0 store (+ db = column sums of B when kind 2 and db != NULL),
 *   epi 1 relu(acc + bias[n]), epi 2 acc * (mask[m][n] > 0).
 * Every operand is dense with the given leading dimension; batch strides are the
 * dense matrix sizes (A shared across the batch when a_shared != 0).
 * precision: low byte = enum mtsac_precision; bits 8-15 = split-K slices for epi 0
 * (0 or 1: no split). */
int mtsac_debug_gemm(int precision, int kind, int epi, int batch, int M, int N, int K, const float* A, int lda, int a_shared,
                     const float* B, int ldb, float* C, int ldc, const float* bias, const float* mask, int ldm,
                     float* db);

/* Time `iters` back-to-back launches of one GEMM on device-resident random operands
 * (allocated once, dense, lda = K or M as the kind requires); writes the mean
 * milliseconds per launch (HIP events on the launch stream). */
int mtsac_debug_gemm_bench(int precision, int kind, int epi, int batch, int M, int N, int K, int iters,
                           double* ms_per_launch);

/* Pre-split-plane GEMM (gemm_x3p.hip): C[M][N] = op(A) . op(B) from host fp32 arrays.
 * a_kmajor: A given as [K][M] (else [M][K]); b_kmajor: B given as [K][N] (else [N][K]).
 * The operands are split into bf16 planes on the device in their stored orientation and
 * multiplied (k-major operands through the transposed LDS read); epi as in mtsac_debug_gemm
 * (bits 8-15: split-K slices for epi 0).  Csum (nullable): the GEMM also writes C's split
 * planes and Csum receives their sum h + m + l. */
int mtsac_debug_gemm_x3p(int epi, int M, int N, int K, const float* A, int a_kmajor, const float* B, int b_kmajor,
                         float* C, const float* bias, const float* mask, float* Csum);
/* Time iters launches of the plane GEMM on device-resident random planes (NT form). */
int mtsac_debug_gemm_x3p_bench(int epi, int batch, int M, int N, int K, int iters, double* ms_per_launch);
/* Select the plane GEMM tile geometry (bits 0-7: 0 = 128x128 k32, 1 = 256x128 k32, 2 = 256x128 k16,
 * 3 = 256x256 k16, 255 = by operand form (default)) and
 * ablation bits for experiments (bits 8-15: plane GEMM, bits 16-23: split GEMM; 0 = normal);
 * returns the old geometry. */
int mtsac_debug_x3p_geo(int geo);

/* Row-major x row-major plane GEMM (gemm_x3f.hip, 16x16x32 MFMA, K padded to 64): per batch entry
 * C[M][N] = epi(A[M][K] . B[N][K]^T); epi 1 bias+ReLU, 2 ReLU mask (bit 8: mask read from the
 * bf16 high plane of `mask`; bit 9: run gemm_x3s.hip, the small-row-count kernel, instead; bit 10:
 * precision bf16, the products on the operands' high planes only; bit 11: split-K by the
 * launcher's choice, with a workspace, as the engine runs task shards);
 * Csum (nullable): sum of the written output planes.  -95 when the kernel does not take the shape. */
int mtsac_debug_gemm_x3f(int epi, int batch, int M, int N, int K, const float* A, const float* B, float* C,
                         const float* bias, const float* mask, float* Csum);
/* Time iters launches of the forward-shaped plane GEMM: which 0 = gemm_x3p (B k-major), 1 = gemm_x3f,
 * -1 = gemm_x3s (-2 / -3: its TI = 7 instance without operand loads / without MFMAs, experiments);
 * epi bits 8-9: outputs 0 = fp32 + planes, 1 = planes only, 2 = fp32 only; bit 10: precision bf16;
 * bit 11: split-K by the launcher's choice (gemm_x3p and gemm_x3f), with a workspace. */
int mtsac_debug_gemm_fwd_bench(int which, int epi, int batch, int M, int N, int K, int iters, double* ms_per_launch);
/* Rows per gemm_x3s tile / 16 (TI, 4..8) the cost model picks for an M x N output, batch entries. */
int mtsac_debug_x3s_ti(int M, int N, int batch);
// DrQ conv channel groups per lane (fwd: output channels, bwd: input channels; 0 = the engine's
// choice); returns the previous fwd | bwd << 8.  Experiments only.
int mtsac_debug_drq_groups(int fwd, int bwd);
// DrQ convolutions on f32 MFMA (experiment, measured slower than the VALU kernels): bit 1 forward,
// 2 data grad, 4 weight grad (default 0 = the VALU kernels).  Returns the previous mask; < 0 queries.
int mtsac_debug_drq_mfma(int mask);
// The pre-round-6 DrQ conv kernels (one lane per pixel, im2col weight grad) instead of the row-tile
// ones: bit 1 forward, 2 data grad, 4 weight grad; bit 8 runs the row-tile kernels at every shape
// (past the measured per-shape choice); bit 16 turns the split2h MFMA convs off, bit 32 runs them at
// every shape they support.  Returns the previous mask; < 0 queries.
int mtsac_debug_drq_legacy(int mask);
// The row-tile conv weight grad's grid cap (> 0 sets, 0 restores the per-shape default, < 0 queries;
// returns the previous).  Engines size their partial buffers at creation: change it only before
// creating one.  Experiments.
int mtsac_debug_drq_wgrad_blocks(int cap);
// Mean microseconds per launch of one DrQ conv pass on random operands: kind 0 forward (ReLU in,
// residual), 1 data gradient (mask, residual), 2 weight-gradient partials.  -22 bad arguments.
int mtsac_debug_drq_conv_bench(int kind, int B, int H, int W, int ci, int co, int iters, double* us_per_launch);

/* Eager update_many overlaps consecutive steps (the next gather and critic(s, a) forward beside
 * the previous actor backward / all-reduce / Adam): on = 1 always, 0 never (whole steps), -1 the
 * default (when the trunk gradients go through a device collective: RCCL or the modelled one).
 * Returns the previous setting.  Tests and experiments. */
struct mtsac_engine;
int mtsac_debug_set_pipeline(struct mtsac_engine* engine, int32_t on);

/* 1 when the engine issues every compute segment on its main stream (the default; the 5-lane
 * form needs MTSAC_LANES=1 and enough hardware queues: GPU_MAX_HW_QUEUES as the process started
 * >= 5 per live engine + 3), else 0. */
int mtsac_debug_lane_mode(struct mtsac_engine* engine);
/* Guard zones (MTSAC_GUARD_BYTES=n in the environment before the engine is created): n bytes of 0xFF
 * around every device allocation.  Returns the number of guards a kernel wrote (0 = intact; -95 when
 * the mode is off); the first few are named in mtsac_last_error. */
int mtsac_debug_check_guards(struct mtsac_engine* engine);
/* Step buffer views (diagnostics): snapshot on/off; read id 0 actor top activations, 1 / 2 their
 * snapshots after the actor forward / the actor-loss pass ([Ma][W]), 3 actor dout ([B][2A]), 4 actor
 * gradient head leaves.  count must equal the buffer's float count. */
int mtsac_debug_snapshot(struct mtsac_engine* engine, int32_t on);
int mtsac_debug_read(struct mtsac_engine* engine, int32_t id, float* dst, int64_t count);
/* the head backward's LDS self-check, tested: the last step's actor head weight pass re-run into a
   scratch output with one cross-wave LDS slot corrupted on purpose; the next mtsac_get_logs /
   mtsac_synchronize must fail (-5, "head backward self-check failed").  Needs a step first. */
int mtsac_debug_head_selfcheck(struct mtsac_engine* engine);
/* Weight planes in the fragment layout (gemm_x3f B operand, engine.cpp Net::bfrag): mode -1 (the
 * default) decides by shape (MTSAC_BFRAG=0 turns it off), 0 / 1 forces it off / allows it, for
 * engines created afterwards.  mtsac_debug_bfrag: bit i actor layer i, bit 8 + i critic layer i. */
int mtsac_debug_set_bfrag(int32_t mode);
int mtsac_debug_bfrag(struct mtsac_engine* engine);
/* on != 0: this engine issues on one stream whatever MTSAC_LANES asks, and is not counted by the
 * lane grant of the other live engines (experiments comparing the two issue forms in one process). */
int mtsac_debug_force_one_stream(struct mtsac_engine* engine, int32_t on);
/* Modelled trunk-gradient collective for one-GPU runs of a task shard: with nranks > 1 the engine
 * takes its sharded path and, at every point where it would call RCCL, issues on the collective
 * stream a delay of 2 (nranks - 1) / nranks * bucket bytes / bus_gbps (GB/s) held by
 * (flags >> 8) & 255 workgroups (0: 8); the data stay as they are (a one-rank sum).  flags bit 0:
 * the bucket reads NaN until the delay is over (a consumer without a stream edge to the
 * collective turns the step into NaN).  nranks = 1 switches it off.  Not with a communicator or hook. */
int mtsac_debug_set_collective_model(struct mtsac_engine* engine, int32_t nranks, double bus_gbps, int32_t flags);

/* Per-launch record of the last timed step (mtsac_set_timing): i < 0 returns the number of
 * records; else dims = {family = GEMM kind, M, N, K, batch} and *ms its duration. */
struct mtsac_engine;
int mtsac_debug_timed_launch(struct mtsac_engine* engine, int32_t i, int32_t* dims, double* ms);

#ifdef __cplusplus
}
#endif
#endif
