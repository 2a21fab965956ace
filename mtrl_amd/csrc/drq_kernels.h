// drq_kernels.h -- launch wrappers of the DrQ-eps device kernels (drq.hip), internal to libmtsac.so.
#pragma once
#include <hip/hip_runtime.h>

namespace mtsac {
namespace drq {

// augment (augmentation.py:101-117), draws given: uint8 [B][C][H][W] -> NHWC [-1, 1] * noise[b],
// edge pad `pad`, crop offsets crop[b] = (along H, along W) in [0, 2 pad]
void augment(const unsigned char* obs, const int* crop, const float* noise, float* out, int B, int C, int H, int W,
             int pad, hipStream_t st);
// the update's encoder input [s | s' | s'] (3B images) from obs and next obs in one launch
void augment3(const unsigned char* obs, const int* crop_o, const float* noise_o, const unsigned char* nobs,
              const int* crop_n, const float* noise_n, float* out, int B, int C, int H, int W, int pad, hipStream_t st);
// MemoryEfficientAtariMultiTaskReplayBuffer.sample rows from the device store (img_bytes % 16 == 0);
// nstore != null: AtariMultiTaskReplayBuffer's separate next_obs array (no guard: pass full = 0)
void atari_sample(const unsigned char* store, const unsigned char* nstore, const int* act, const float* rew,
                  const float* done, const float* trunc, const double* minmax, const int* idx, long long cap, int T,
                  int n, int img_bytes, int nstep, int full, int pos, int guard, double eps, unsigned char* obs,
                  unsigned char* nobs, int* act_out, float* rew_out, float* done_out, float* trunc_out, int* task_out,
                  hipStream_t st);
// sample_unbalanced rows: row b = (slot slots[b], task tasks[b]), both drawn on the host
void atari_sample_rows(const unsigned char* store, const unsigned char* nstore, const int* act, const float* rew,
                       const float* done, const float* trunc, const double* minmax, const long long* slots,
                       const int* tasks, int rows, long long cap, int T, int img_bytes, int nstep, double eps, unsigned char* obs,
                       unsigned char* nobs, int* act_out, float* rew_out, float* done_out, float* trunc_out,
                       int* task_out, hipStream_t st);
// fresh augmentation draws for obs and next_obs from (seed, ctr): crops in [0, 2 pad), intensity
// 1 + 0.05 clip(N(0, 1), -2, 2)
void aug_draw(unsigned long long seed, unsigned long long ctr, int B, int pad, int* crop_o, float* noise_o,
              int* crop_n, float* noise_n, hipStream_t st);
bool conv_supported(int ci, int co);
extern int g_drq_fwd_g, g_drq_bwd_g;  // conv channel groups per lane, 0: the engine's choice (experiments)
extern int g_drq_mfma;  // f32-MFMA convs (experiment): bit 1 forward, 2 data grad, 4 weight grad (default 0)
// the pre-round-6 conv kernels (one lane per pixel; im2col weight grad) instead of the row-tile
// ones: bit 1 forward, 2 data grad, 4 weight grad; bit 8: the row-tile kernels at every shape (past
// the measured per-shape choice) where bits 1-4 are clear; bit 16: no split2h MFMA convs; bit 32: the
// split2h MFMA convs at every shape they support (default 0; tests and A/B)
extern int g_drq_legacy;
extern int g_drq_wg_blocks;  // the row-tile weight grad's grid cap (experiments; set before an engine exists)
double conv_bench(int kind, int B, int H, int W, int ci, int co, int iters);
// 3x3 / stride 1 / SAME on NHWC, kernel [3][3][ci][co]; relu_in applies ReLU to the input, res
// (nullable) is added to the output.  w2 / bias2 (nullable): images [B1, B) use that second
// parameter set (one launch over the online and the target passes)
void conv_fwd(const float* in, const float* w, const float* bias, const float* res, float* out, int B, int H, int W,
              int ci, int co, bool relu_in, hipStream_t st, const float* w2 = nullptr, const float* bias2 = nullptr,
              int B1 = -1);
// din = conv^T(dout) * [mask > 0] (mask nullable) + dres (nullable)
void conv_bwd_data(const float* dout, const float* w, const float* mask, const float* dres, float* din, int B, int H,
                   int W, int ci, int co, hipStream_t st);
// the row-tile weight-gradient kernel's geometry: tiles of R image rows (tiles = B ceil(H / R)), LDS
// row stride SR floats, magic = ceil(2^32 / W) (q / W = umulhi(q, magic) for the q < R W it divides)
struct WgGeo {
  int H, W, R, SR, tiles;
  unsigned magic;
};
int conv_wgrad_blocks(int B, int H, int W, int ci, int co);
// the row-tile forward / data-gradient kernels' geometry: n tiles of R rows per image, LDS row
// stride SR floats, magic = ceil(2^32 / W), magic2 = ceil(2^32 / (W + 2))
struct ConvGeo {
  int H, W, R, SR, n;
  unsigned magic, magic2;
};
// dw [3][3][ci][co], db [co] of a conv whose input is act(in); part: conv_wgrad_blocks(...) x
// (9 ci co + co) floats
// defer_sum: leave the partials for one sum_parts_multi launch over every conv of the backward
void conv_wgrad(const float* in, const float* dout, float* part, float* dw, float* db, int B, int H, int W, int ci,
                int co, bool relu_in, hipStream_t st, bool defer_sum = false);
// one conv's partial sums: part[G][n] -> dw[0, nw), db[0, n - nw); blocks [blk0, blk0 + sum_parts_blocks)
struct SumSeg {
  const float* part;
  float *dw, *db;
  int G, n, nw, blk0;
};
int sum_parts_blocks(int ci, int co);
void sum_parts_multi(const SumSeg* segs, int nseg, int blocks, hipStream_t st);
// max pool 3x3 / stride 2 / SAME (out (H + 1) / 2), argmax tap per output
void maxpool_fwd(const float* in, float* out, unsigned char* arg, int B, int H, int W, int C, hipStream_t st);
void maxpool_bwd(const float* dout, const unsigned char* arg, float* din, int B, int H, int W, int C, hipStream_t st);
// feat[b] = [relu(enc[b]) | normalised emb[task[(r0 + b) % tmod]]]
void concat_feat(const float* enc, int nenc, const float* emb, int D, const int* task, int r0, int tmod, float* feat,
                 int ldf, int B, hipStream_t st);
// LayerNorm over F columns of (x + xb) (xb nullable), y = ln * scale + bias (ReLU when relu)
void ln_fwd(const float* x, const float* xb, int ldx, int F, const float* scale, const float* bias, float eps,
            float* y, int ldy, float* xhat, float* rstd, int B, bool relu, hipStream_t st);
void ln_bwd(const float* dy, int lddy, const float* y, int ldy, const float* xhat, const float* rstd,
            const float* scale, int F, float* dx, int lddx, float* dscale, float* dbias, int B, bool relu,
            hipStream_t st);
void colsum_rows(const float* x, int ld, int F, int B, float* out, hipStream_t st);
// head output hc[b][ldh] = [adv (A Z) | val (Z)] before bias (hb): C51 target m[b][Z]
void c51_target(const float* hc_on, const float* hc_tg, int ldh, const float* hb_on, const float* hb_tg, int A, int Z,
                const float* rew, const float* done, float gamma_n, float vmin, float vmax, float* m, int* a_next,
                int B, hipStream_t st);
// expected Q per action: q[b][a] = softmax_z(logit[b][a]) . support
void q_values(const float* hc, int ldh, const float* hb, int A, int Z, float vmin, float vmax, float* q, int B,
              hipStream_t st);
void c51_loss(const float* hc, int ldh, const float* hb, int A, int Z, const int* act, const float* m, float* dh,
              float* loss_b, float* logit_b, int B, hipStream_t st);
void embed_bwd(const float* dfeat, int ldf, int off, const float* emb, int D, const int* task, int B, int T,
               float* demb, hipStream_t st);
void enc_grad(const float* dfeat, int ldf, const float* enc, int nenc, float* denc, int B, hipStream_t st);
// optax.adamw + Polyak over a flat buffer; part[2 G]: sum g^2, sum p_pre^2 per block; returns G
int adamw(float* p, float* mu, float* nu, const float* g, float* tgt, long long n, float lr, float b1, float b2,
          float eps, float wd, float tau, int count, float* part, int max_blocks, hipStream_t st);
// logs = [mean online logit, |g|, |p_pre|, mean loss]
void drq_logs(const float* part, int G, const float* loss_b, const float* logit_b, int B, int Z, float* logs,
              hipStream_t st);

// compute_weights (drqeps.py:353-482): one gradient from the internal layout to flax ravel order
// through the (f, i, n, ld, rows) segment table (entries x 5 int64 on the device)
void flax_gather(const float* g, const long long* map, int entries, long long max_n, float* out, hipStream_t st);
// project_grad (drqeps.py:428-448) of T <= jl_max_tasks() rows of G [T][ldg] at once:
// out[t][j] = sum_k G[t][k] N(k, j) / sqrt(D), N = jax.random.normal(PRNGKey(seed + k / chunk),
// (chunk, D))[k % chunk][j] regenerated on the fly (threefry2x32, partitionable); part holds
// jl_part_floats(P, D) floats
int jl_max_tasks();
long long jl_part_floats(long long P, int D);
void jl_project(const float* G, long long ldg, int T, long long P, int D, long long chunk, int seed, float* part,
                float* out, long long ldo, hipStream_t st);
}  // namespace drq
}  // namespace mtsac
