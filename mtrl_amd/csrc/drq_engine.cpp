// drq_engine.cpp -- the DrQ-eps update engine behind include/drq.h.
//
// One update (DrQ.update + _update_inner, mtrl/rl/algorithms/drqeps.py:268-343) on the engine's
// stream: augment obs / next_obs; online and target forwards at s' -> greedy action and the C51
// target m; the online forward at s saving its activations; cross entropy at the taken action;
// the backward (dueling head -> LayerNorms -> embedding and the IMPALA stacks in reverse); AdamW,
// Polyak, logs.  Dense layers run on gemm_f32 (exact fp32), everything else on drq.hip.
//
// Parameters live in an internal layout (each leaf 256-B aligned; Dense_1 (advantage) and Dense_2
// (value) side by side as one [H][A Z + Z (+pad)] matrix so the head is one GEMM); set/get
// translate from / to the flax ravel order of oracle/drq.py:param_spec().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/drq.h"
#include "drq_kernels.h"
#include "kernels.h"

using namespace mtsac;

extern "C" int pcg_jump_table(unsigned long long* out);  // engine.cpp: numpy PCG64 jumps

namespace {

thread_local std::string g_err;

int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc;
}

long long al(long long x) { return (x + 63) / 64 * 64; }

struct Stack {
  int hin, ci, co, ho;
  long long cb[5], cw[5];  // bias / kernel offsets of Conv_0..Conv_4 (internal layout)
  // saved activations of the online pass at s (stack 0's input: the augmented obs, xin_own)
  float* xin_own = nullptr;
  float* conv0 = nullptr;  // [B][hin][hin][co] pre-pool
  unsigned char* arg = nullptr;
  float* c[3] = {};        // block inputs / output, [B][ho][ho][co]
  float* r[2] = {};        // residual blocks' inner pre-activations
};

}  // namespace

struct drq_engine {
  drq_config cfg{};
  hipStream_t st = nullptr;
  int B = 0, A = 0, Z = 0, T = 0, D = 0, H = 0, F = 0, NENC = 0, NC = 0, count = 0;
  float gamma_n = 0.f;
  Stack stk[3];
  long long off_emb = 0, off_ln1b = 0, off_ln1s = 0, off_w0 = 0, off_b0 = 0, off_ln2b = 0, off_ln2s = 0, off_wc = 0,
            off_bc = 0, n_int = 0, n_flax = 0;
  // flax order -> internal: (flax offset, internal offset, count, row stride in the internal
  // matrix (0 = contiguous), rows)
  struct Map {
    long long f, i, n, ld, rows;
  };
  std::vector<Map> map;
  float *p = nullptr, *g = nullptr, *mu = nullptr, *nu = nullptr, *tgt = nullptr;
  // inputs
  unsigned char *obs_u8 = nullptr, *nobs_u8 = nullptr;
  int task_mod = 1 << 30;  // head rows r read task[r % task_mod] (the update's 3B rows: B)
  int *act = nullptr, *task = nullptr, *crop_o = nullptr, *crop_n = nullptr, *a_next = nullptr;
  float *rew = nullptr, *done = nullptr, *noise_o = nullptr, *noise_n = nullptr;
  float* nobs = nullptr;  // augmented next_obs
  // head activations
  float *feat = nullptr, *xhat1 = nullptr, *rstd1 = nullptr, *ln1 = nullptr, *z1 = nullptr, *xhat2 = nullptr,
        *rstd2 = nullptr, *h2 = nullptr, *hc = nullptr, *hc_on = nullptr, *hc_tg = nullptr, *m = nullptr;
  // backward
  float *dhc = nullptr, *dh2 = nullptr, *dz1 = nullptr, *dln1 = nullptr, *dfeat = nullptr;
  float *ga = nullptr, *gb = nullptr, *gc = nullptr;  // conv activation grads (largest tensor)
  float* wparts[3][5] = {};  // per conv (stack, conv index): its weight-grad partials
  drq::SumSeg* d_segs = nullptr;
  int seg_blocks = 0;
  float *ws = nullptr, *part = nullptr, *loss_b = nullptr, *logit_b = nullptr, *logs = nullptr;
  long long ws_floats = 0;
  std::vector<void*> allocs;
  // ---- device replay buffer (MemoryEfficientAtariMultiTaskReplayBuffer)
  long long cap = 0, img = 0, pos = 0;
  int full = 0, ns_pos = 0, ns_count = 0, n_per_task = 0;
  unsigned char* store = nullptr;
  unsigned char* nstore = nullptr;  // buffer kind 1: next_obs [cap][T][img]
  int* b_act = nullptr;
  float *b_rew = nullptr, *b_done = nullptr, *b_trunc = nullptr, *trunc = nullptr;
  double* d_minmax = nullptr;
  PcgDev* rng = nullptr;
  unsigned long long* jump = nullptr;
  int* idx = nullptr;
  static constexpr int ROWS_STEPS = 64;  // host-drawn rows staged per upload (sample_rows_update)
  long long* r_slot = nullptr;           // [ROWS_STEPS][B]
  int* r_task = nullptr;
  unsigned long long aug_seed = 0, aug_ctr = 0;
  // ---- compute_weights: per-task gradients in flax order [slots][n_flax], the segment table
  long long* d_map = nullptr;
  long long map_max = 0;
  float* tg = nullptr;
  int tg_slots = 0;
  float* jl_part = nullptr;
  long long jl_part_n = 0;
  float* jl_out = nullptr;
  long long jl_out_n = 0;
  std::vector<unsigned char> ns_obs, ns_next;  // [nstep][T][img]
  std::vector<int> ns_act;
  std::vector<float> ns_rew, ns_trunc, ns_done;  // [nstep][T]
  std::vector<double> minmax;                    // [2][T]: min, max

  // (re)allocate a lazily sized buffer
  template <class T_>
  int realloc_buf(T_** ptr, long long& have, long long n) {
    if (n <= have) return 0;
    if (*ptr) {
      if (hipStreamSynchronize(st) != hipSuccess) return fail(-5, "stream sync failed");
      allocs.erase(std::remove(allocs.begin(), allocs.end(), (void*)*ptr), allocs.end());
      (void)hipFree(*ptr);
      *ptr = nullptr;
    }
    int rc = alloc(ptr, n);
    if (!rc) have = n;
    return rc;
  }

  template <class T_>
  int alloc(T_** ptr, long long n) {
    void* q = nullptr;
    if (hipMalloc(&q, sizeof(T_) * (size_t)std::max(n, 1LL)) != hipSuccess) return fail(-12, "hipMalloc failed");
    // zeroed and COMPLETE before returning: callers fill some buffers right away with a plain
    // hipMemcpy (segment tables), which is not ordered after work on the non-blocking engine
    // stream -- an asynchronous memset here could land after the copy and zero the table
    if (hipMemsetAsync(q, 0, sizeof(T_) * (size_t)std::max(n, 1LL), st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail(-5, "memset");
    allocs.push_back(q);
    *ptr = static_cast<T_*>(q);
    return 0;
  }

  // ------------------------------------------------------------------ forward
  // ImpalaDQN at params P on augmented images X -> combined head output out[B][NC] (no bias);
  // the saved activations of the backward are the first B rows of the pass (the activation buffers
  // hold 3B rows: the update's pass covers online s, online s' and target s' at once)
  // rows: B (<= 3 x the batch, see the buffers); P2 (nullable): rows [B1, B) run at params P2
  void forward_rows(const float* P, const float* X, float* out, int B, const float* P2 = nullptr, int B1 = -1) {
    if (P2 == nullptr) B1 = B;
    const float* Q2 = P2 ? P2 : P;
    const float* x = X;
    for (int s = 0; s < 3; ++s) {
      Stack& k = stk[s];
      conv_fwd_t(x, P, Q2, k.cw[0], k.cb[0], nullptr, k.conv0, B, B1, k.hin, k.ci, k.co, false);
      drq::maxpool_fwd(k.conv0, k.c[0], k.arg, B, k.hin, k.hin, k.co, st);
      for (int b = 0; b < cfg_blocks(); ++b) {
        conv_fwd_t(k.c[b], P, Q2, k.cw[1 + 2 * b], k.cb[1 + 2 * b], nullptr, k.r[b], B, B1, k.ho, k.co, k.co, true);
        conv_fwd_t(k.r[b], P, Q2, k.cw[2 + 2 * b], k.cb[2 + 2 * b], k.c[b], k.c[b + 1], B, B1, k.ho, k.co, k.co, true);
      }
      x = k.c[2];
    }
    head_rows(P, 0, B1, out);
    if (B1 < B) head_rows(Q2, B1, B - B1, out);
  }
  // the dense head of rows [r0, r0 + n) at params P
  void head_rows(const float* P, int r0, int n, float* out) {
    const long long r = r0;
    // the update's 3B rows [s | s' | s'] share the batch's B task ids
    drq::concat_feat(stk[2].c[2] + r * NENC, NENC, P + off_emb, D, task, r0, task_mod, feat + r * F, F, n, st);
    drq::ln_fwd(feat + r * F, nullptr, F, F, P + off_ln1s, P + off_ln1b, cfg.ln_eps, ln1 + r * F, F, xhat1 + r * F,
                rstd1 + r, n, false, st);
    gemm_store(ln1 + r * F, F, P + off_w0, H, z1 + r * H, H, n, H, F, GEMM_NN);
    drq::ln_fwd(z1 + r * H, P + off_b0, H, H, P + off_ln2s, P + off_ln2b, cfg.ln_eps, h2 + r * H, H, xhat2 + r * H,
                rstd2 + r, n, true, st);
    gemm_store(h2 + r * H, H, P + off_wc, NC, out + r * NC, NC, n, NC, H, GEMM_NN);
  }
  int cfg_blocks() const { return 2; }

  // ---- per-launch timing of the conv forward family (bench.py's roofline): HIP events on the
  // engine stream around each launch of every 8th update (event records cost host time on a
  // launch-dense step), algorithmic flops 2 B H W 9 ci co
  bool timing = false;
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  double t_flops = 0;
  long long t_launches = 0;
  // conv (weights at offset cw, bias at cb) of images [0, B1) at params P and [B1, Bn) at P2
  void conv_fwd_t(const float* in, const float* P, const float* P2, long long cw, long long cb, const float* res,
                  float* out, int Bn, int B1, int Hh, int ci, int co, bool relu_in) {
    const int Ww = Hh;
    hipEvent_t a = nullptr, b = nullptr;
    if (timing && count % 8 == 0) {
      while (ev.size() < ev_used + 2) {
        hipEvent_t x;
        if (hipEventCreate(&x) != hipSuccess) break;
        ev.push_back(x);
      }
      if (ev.size() >= ev_used + 2) {
        a = ev[ev_used];
        b = ev[ev_used + 1];
        ev_used += 2;
        (void)hipEventRecord(a, st);
      }
    }
    drq::conv_fwd(in, P + cw, P + cb, res, out, Bn, Hh, Ww, ci, co, relu_in, st, P2 + cw, P2 + cb, B1);
    if (a) {
      (void)hipEventRecord(b, st);
      t_flops += 2.0 * Bn * Hh * Ww * 9.0 * ci * co;
      ++t_launches;
    }
  }

  // expected Q of the online network on n (<= batch) staged observations (rollout actions)
  void q_values(int n, float* q) {
    drq::augment(obs_u8, crop_o, noise_o, stk[0].xin_own, n, cfg.in_ch, cfg.hw, cfg.hw, 4, st);
    forward_rows(p, stk[0].xin_own, hc_on, n);
    drq::q_values(hc_on, NC, p + off_bc, A, Z, cfg.v_min, cfg.v_max, q, n, st);
  }

  // the dense layers' GEMMs: exact fp32 FMAs (gemm_f32), or with MTSAC_DRQ_DENSE=x3 the
  // fp32-accurate split-bf16 MFMA form (gemm_x3: same contract, error that of an fp32 GEMM)
  void dense(const GemmParams& gp, GemmKind kind) {
    static const bool x3 = [] {
      const char* e = getenv("MTSAC_DRQ_DENSE");
      return e && std::string(e) == "x3";
    }();
    if (x3) gemm_x3(gp, kind, EPI_STORE, 1, st);
    else gemm_f32(gp, kind, EPI_STORE, 1, st);
  }

  // C[M][N] = A . op(B) with split-K over the few row tiles a batch of 256 gives (EPI_STORE)
  void gemm_store(const float* Aop, int lda, const float* Bop, int ldb, float* C, int ldc, int M, int N, int K,
                  GemmKind kind) {
    GemmParams gp{};
    gp.A = Aop; gp.lda = lda;
    gp.B = Bop; gp.ldb = ldb;
    gp.C = C; gp.ldc = ldc;
    gp.M = M; gp.N = N; gp.K = K;
    gp.splits = gemm_splits(M, N, K, 1);
    gp.ws = ws;
    dense(gp, kind);
  }

  void wgrad_gemm(const float* Aop, int lda, const float* Bop, int ldb, float* C, float* db, int M, int N) {
    GemmParams gp{};
    gp.A = Aop; gp.lda = lda;  // [K = B][M]
    gp.B = Bop; gp.ldb = ldb;  // [K = B][N]
    gp.C = C; gp.ldc = N;
    gp.db = db;
    gp.M = M; gp.N = N; gp.K = B;
    gp.splits = gemm_splits(M, N, B, 1);
    gp.ws = ws;
    dense(gp, GEMM_TN);
  }

  // ------------------------------------------------------------------ replay
  // add (buffers.py:1138-1186): n-step ring on the host, the aggregated transition to the device
  int buffer_add(const unsigned char* o, const unsigned char* no, const int* a, const float* r, const float* tr,
                 const float* d) {
    const int n = cfg.nstep;
    const size_t row = (size_t)T * img;
    const int sl = ns_pos;
    std::memcpy(&ns_obs[sl * row], o, row);
    std::memcpy(&ns_next[sl * row], no, row);
    for (int t = 0; t < T; ++t) {
      ns_act[sl * T + t] = a[t];
      ns_rew[sl * T + t] = r[t];
      ns_trunc[sl * T + t] = tr[t];
      ns_done[sl * T + t] = d[t];
    }
    ns_pos = (sl + 1) % n;
    ns_count = std::min(ns_count + 1, n);
    if (ns_count < n) return 0;
    // _get_nstep_info (buffers.py:1048-1080): float32 arithmetic in the reference's order
    const int oldest = ns_pos, newest = (ns_pos - 1 + n) % n;
    std::vector<float> rw(&ns_rew[newest * T], &ns_rew[newest * T] + T), dn(&ns_done[newest * T], &ns_done[newest * T] + T);
    std::vector<int> src(T, newest);  // which ring slot's next_obs each task takes
    const float g = cfg.gamma;
    for (int k = 1; k < n; ++k) {
      const int i = ((ns_pos - 1 - k) % n + n) % n;
      for (int t = 0; t < T; ++t) {
        float v = rw[t] * g;
        v = v * (1.0f - ns_done[i * T + t]);
        rw[t] = v + ns_rew[i * T + t];
        if (ns_done[i * T + t] > 0.0f) {
          src[t] = i;
          dn[t] = ns_done[i * T + t];
        }
      }
    }
    const long long p = pos, pn = nstore ? pos : (pos + n) % cap;
    std::vector<unsigned char> nxt(row);
    for (int t = 0; t < T; ++t) std::memcpy(&nxt[(size_t)t * img], &ns_next[(size_t)src[t] * row + (size_t)t * img], img);
    if (hipMemcpyAsync(store + (size_t)p * row, &ns_obs[(size_t)oldest * row], row, hipMemcpyHostToDevice, st) !=
            hipSuccess ||
        hipMemcpyAsync((nstore ? nstore : store) + (size_t)pn * row, nxt.data(), row, hipMemcpyHostToDevice, st) !=
            hipSuccess ||
        hipMemcpyAsync(b_act + p * T, &ns_act[oldest * T], sizeof(int) * T, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b_rew + p * T, rw.data(), sizeof(float) * T, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b_done + p * T, dn.data(), sizeof(float) * T, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b_trunc + p * T, &ns_trunc[oldest * T], sizeof(float) * T, hipMemcpyHostToDevice, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)  // the host staging above is stack / ring memory
      return fail(-5, "buffer upload failed");
    if (cfg.normalize_rewards)
      for (int t = 0; t < T; ++t) {
        minmax[t] = std::min(minmax[t], (double)rw[t]);
        minmax[T + t] = std::max(minmax[T + t], (double)rw[t]);
      }
    pos = (p + 1) % cap;
    if (pos == 0) full = 1;
    return 0;
  }

  // sample (buffers.py:1188-1227) into the staged batch
  int sample() {
    if (n_per_task < 1 || B % T != 0) return fail(-22, "balanced sample: batch % num_tasks must be 0");
    const int n = n_per_task, guard = cfg.nstep + 6;
    // kind 1: integers(0, max(pos or capacity, n)) (buffers.py:863-869)
    const long long high = nstore ? std::max(full ? cap : pos, (long long)n)
                                  : full ? cap - guard : std::max(pos - cfg.nstep, 1LL);
    replay_indices_high(rng, jump, high, n, idx, st);
    if (cfg.normalize_rewards &&
        hipMemcpyAsync(d_minmax, minmax.data(), sizeof(double) * 2 * T, hipMemcpyHostToDevice, st) != hipSuccess)
      return fail(-5, "reward stats upload failed");
    drq::atari_sample(store, nstore, b_act, b_rew, b_done, b_trunc, cfg.normalize_rewards ? d_minmax : nullptr, idx,
                      cap, T, n, (int)img, cfg.nstep, nstore ? 0 : full, (int)pos, guard, 1e-8, obs_u8, nobs_u8, act,
                      rew, done, trunc, task, st);
    return 0;
  }

  // sample_unbalanced (buffers.py:1230-1279) with the rows drawn by the caller: rows [s][B] at
  // slots / tasks already on the device
  int sample_rows(const long long* slots, const int* tasks) {
    if (cfg.normalize_rewards &&
        hipMemcpyAsync(d_minmax, minmax.data(), sizeof(double) * 2 * T, hipMemcpyHostToDevice, st) != hipSuccess)
      return fail(-5, "reward stats upload failed");
    drq::atari_sample_rows(store, nstore, b_act, b_rew, b_done, b_trunc, cfg.normalize_rewards ? d_minmax : nullptr,
                           slots, tasks, B, cap, T, (int)img, cfg.nstep, 1e-8, obs_u8, nobs_u8, act, rew, done, trunc,
                           task, st);
    return 0;
  }

  // checked upload of `steps` host-drawn row sets into r_slot / r_task (stream ordered)
  int upload_rows(const long long* slots, const int* tasks, int steps) {
    const long long n = (long long)steps * B;
    for (long long i = 0; i < n; ++i)
      if (slots[i] < 0 || slots[i] >= cap || tasks[i] < 0 || tasks[i] >= T)
        return fail(-22, "row " + std::to_string(i) + ": slot or task out of range");
    if (hipMemcpyAsync(r_slot, slots, sizeof(long long) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(r_task, tasks, sizeof(int) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)  // the caller's arrays may go away on return
      return fail(-5, "row upload failed");
    return 0;
  }

  void draw_aug() { drq::aug_draw(aug_seed, aug_ctr++, B, 4, crop_o, noise_o, crop_n, noise_n, st); }

  // ------------------------------------------------------------------ one update on the staged batch
  void step() {
    grad_pass();
    ++count;
    const int G = drq::adamw(p, mu, nu, g, tgt, n_int, cfg.lr, cfg.b1, cfg.b2, cfg.eps, cfg.weight_decay, cfg.tau,
                             count, part, 1024, st);
    drq::drq_logs(part, G, loss_b, logit_b, B, Z, logs, st);
  }

  // the loss gradient of the staged batch into g (drqeps.py:268-308 up to the optimizer)
  void grad_pass() {
    const int C0 = cfg.in_ch;
    // ONE pass over the 3B images [s | s' | s'] (nobs = xin_own + B images, written with its copy
    // by one augmentation launch): online params for the first 2B, target params for the last B
    // (per-image arithmetic does not depend on the batch).  Its first B rows are the activations
    // the backward reads; head rows [B, 2B) are the online head at s', [2B, 3B) the target's.
    drq::augment3(obs_u8, crop_o, noise_o, nobs_u8, crop_n, noise_n, stk[0].xin_own, B, C0, cfg.hw, cfg.hw, 4, st);
    task_mod = B;
    forward_rows(p, stk[0].xin_own, hc, 3 * B, tgt, 2 * B);
    task_mod = 1 << 30;
    drq::c51_target(hc + (long long)B * NC, hc + 2LL * B * NC, NC, p + off_bc, tgt + off_bc, A, Z, rew, done, gamma_n,
                    cfg.v_min, cfg.v_max, m, a_next, B, st);
    drq::c51_loss(hc, NC, p + off_bc, A, Z, act, m, dhc, loss_b, logit_b, B, st);
    // ---- head backward
    wgrad_gemm(h2, H, dhc, NC, g + off_wc, g + off_bc, H, NC);
    gemm_store(dhc, NC, p + off_wc, NC, dh2, H, B, H, NC, GEMM_NT);  // Wc as [N = H][K = NC]
    drq::ln_bwd(dh2, H, h2, H, xhat2, rstd2, p + off_ln2s, H, dz1, H, g + off_ln2s, g + off_ln2b, B, true, st);
    drq::colsum_rows(dz1, H, H, B, g + off_b0, st);
    wgrad_gemm(ln1, F, dz1, H, g + off_w0, nullptr, F, H);
    gemm_store(dz1, H, p + off_w0, H, dln1, F, B, F, H, GEMM_NT);  // W0 as [N = F][K = H]
    drq::ln_bwd(dln1, F, nullptr, 0, xhat1, rstd1, p + off_ln1s, F, dfeat, F, g + off_ln1s, g + off_ln1b, B, false, st);
    drq::embed_bwd(dfeat, F, NENC, p + off_emb, D, task, B, T, g + off_emb, st);
    // ---- encoder backward, stacks in reverse
    // dc: grad wrt the current block / stack output; dr: scratch; dn: the grad being produced
    float *dc = ga, *dr = gb, *dn = gc;
    drq::enc_grad(dfeat, F, stk[2].c[2], NENC, dc, B, st);
    for (int s = 2; s >= 0; --s) {
      Stack& k = stk[s];
      for (int b = 1; b >= 0; --b) {  // c[b + 1] = conv_k2(relu(r[b])) + c[b], r[b] = conv_k1(relu(c[b]))
        const int k2 = 2 + 2 * b, k1 = 1 + 2 * b;
        drq::conv_wgrad(k.r[b], dc, wparts[s][k2], g + k.cw[k2], g + k.cb[k2], B, k.ho, k.ho, k.co, k.co, true, st, true);
        drq::conv_bwd_data(dc, p + k.cw[k2], k.r[b], nullptr, dr, B, k.ho, k.ho, k.co, k.co, st);
        drq::conv_wgrad(k.c[b], dr, wparts[s][k1], g + k.cw[k1], g + k.cb[k1], B, k.ho, k.ho, k.co, k.co, true, st, true);
        drq::conv_bwd_data(dr, p + k.cw[k1], k.c[b], dc, dn, B, k.ho, k.ho, k.co, k.co, st);
        std::swap(dc, dn);
      }
      drq::maxpool_bwd(dc, k.arg, dn, B, k.hin, k.hin, k.co, st);  // dn: grad wrt conv0's output
      const float* xin = s == 0 ? stk[0].xin_own : stk[s - 1].c[2];
      drq::conv_wgrad(xin, dn, wparts[s][0], g + k.cw[0], g + k.cb[0], B, k.hin, k.hin, k.ci, k.co, false, st, true);
      if (s > 0) drq::conv_bwd_data(dn, p + k.cw[0], nullptr, nullptr, dc, B, k.hin, k.hin, k.ci, k.co, st);
    }
    // every conv's weight / bias gradient from its partials, one launch (the segment table)
    drq::sum_parts_multi(d_segs, 15, seg_blocks, st);
  }
};

namespace {

int copy_in(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!src) return fail(-22, "null input pointer");
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st) == hipSuccess ? 0 : fail(-5, "hipMemcpyAsync");
}

}  // namespace

extern "C" {

const char* drq_last_error(void) { return g_err.c_str(); }

int drq_create(const drq_config* c, int device, drq_engine** out) {
  if (!c || !out) return fail(-22, "null argument");
  *out = nullptr;
  if (c->num_tasks < 1 || c->n_actions < 1 || c->n_atoms < 2 || c->n_atoms > 64 || c->batch < 1 || c->hw < 4 ||
      c->scale < 1 || c->embed_dim < 1 || c->embed_dim > 64 || c->n_hidden < 4)
    return fail(-22, "bad drq_config");
  // 32-bit indices in the conv / pool kernels, over the update's 3B-image forward pass
  if (3LL * c->batch * c->hw * c->hw * 16 * c->scale >= (1LL << 31))
    return fail(-22, "batch x hw x hw x channels must stay below 2^31");
  if (hipSetDevice(device) != hipSuccess) return fail(-19, "hipSetDevice failed");
  drq_engine* e = new drq_engine();
  e->cfg = *c;
  auto bad = [&](int rc) {
    drq_destroy(e);
    return rc;
  };
  if (hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) != hipSuccess) return bad(fail(-5, "stream"));
  const int B = e->B = c->batch;
  e->A = c->n_actions;
  e->Z = c->n_atoms;
  e->T = c->num_tasks;
  e->D = c->embed_dim;
  e->H = c->n_hidden * c->scale;
  e->gamma_n = (float)std::pow((double)c->gamma, (double)c->nstep);
  // layout: stacks
  const int chans[3] = {8 * c->scale, 16 * c->scale, 16 * c->scale};
  int h = c->hw, ci = c->in_ch;
  long long o = 0;
  for (int s = 0; s < 3; ++s) {
    Stack& k = e->stk[s];
    k.hin = h;
    k.ci = ci;
    k.co = chans[s];
    k.ho = (h + 1) / 2;
    if (!drq::conv_supported(k.ci, k.co) || !drq::conv_supported(k.co, k.co)) {
      delete e;
      return fail(-95, "conv channel counts not instantiated (scale 1, in_ch 4)");
    }
    for (int q = 0; q < 5; ++q) {
      const int cin = q == 0 ? k.ci : k.co;
      k.cb[q] = o;
      o = al(o + k.co);
      k.cw[q] = o;
      o = al(o + 9LL * cin * k.co);
    }
    h = k.ho;
    ci = k.co;
  }
  e->NENC = e->stk[2].ho * e->stk[2].ho * e->stk[2].co;
  e->F = e->NENC + e->D;
  if (e->F % 4 != 0 || e->H % 4 != 0) {
    delete e;
    return fail(-95, "feature / hidden widths must be multiples of 4");
  }
  e->NC = (int)((e->A * e->Z + e->Z + 3) / 4 * 4);
  const int F = e->F, H = e->H, NC = e->NC, A = e->A, Z = e->Z;
  e->off_emb = o; o = al(o + (long long)e->T * e->D);
  e->off_ln1b = o; o = al(o + F);
  e->off_ln1s = o; o = al(o + F);
  e->off_w0 = o; o = al(o + (long long)F * H);
  e->off_b0 = o; o = al(o + H);
  e->off_ln2b = o; o = al(o + H);
  e->off_ln2s = o; o = al(o + H);
  e->off_wc = o; o = al(o + (long long)H * NC);
  e->off_bc = o; o = al(o + NC);
  e->n_int = o;
  // flax ravel order (oracle/drq.py:param_spec)
  long long f = 0;
  auto add = [&](long long i, long long n, long long ld = 0, long long rows = 1) {
    e->map.push_back({f, i, n, ld, rows});
    f += n * rows;
  };
  add(e->off_b0, H);                       // Dense_0/bias
  add(e->off_w0, (long long)F * H);        // Dense_0/kernel
  add(e->off_bc, (long long)A * Z);        // Dense_1/bias (advantage)
  add(e->off_wc, (long long)A * Z, NC, H); // Dense_1/kernel rows
  add(e->off_bc + (long long)A * Z, Z);    // Dense_2/bias (value)
  add(e->off_wc + (long long)A * Z, Z, NC, H);
  add(e->off_ln2b, H);
  add(e->off_ln2s, H);
  for (int s = 0; s < 3; ++s)
    for (int q = 0; q < 5; ++q) {
      const Stack& k = e->stk[s];
      add(k.cb[q], k.co);
      add(k.cw[q], 9LL * (q == 0 ? k.ci : k.co) * k.co);
    }
  add(e->off_ln1b, F);
  add(e->off_ln1s, F);
  add(e->off_emb, (long long)e->T * e->D);
  e->n_flax = f;
  int rc;
  {
    std::vector<long long> tab;
    for (const auto& mp : e->map) {
      tab.insert(tab.end(), {mp.f, mp.i, mp.n, mp.ld, mp.rows});
      e->map_max = std::max(e->map_max, mp.n * mp.rows);
    }
    if ((rc = e->alloc(&e->d_map, (long long)tab.size())) ||
        hipMemcpy(e->d_map, tab.data(), sizeof(long long) * tab.size(), hipMemcpyHostToDevice) != hipSuccess)
      return bad(rc ? rc : fail(-5, "segment table upload"));
  }
  for (float** q : {&e->p, &e->g, &e->mu, &e->nu, &e->tgt})
    if ((rc = e->alloc(q, e->n_int))) return bad(rc);
  const long long img = (long long)B * c->in_ch * c->hw * c->hw;
  if ((rc = e->alloc(&e->obs_u8, img)) || (rc = e->alloc(&e->nobs_u8, img))) return bad(rc);
  for (int** q : {&e->act, &e->a_next})
    if ((rc = e->alloc(q, B))) return bad(rc);
  if ((rc = e->alloc(&e->task, 3 * B))) return bad(rc);  // [task | task | task]: the pass over s, s', s'
  if ((rc = e->alloc(&e->crop_o, 2 * B)) || (rc = e->alloc(&e->crop_n, 2 * B))) return bad(rc);
  for (float** q : {&e->rew, &e->done, &e->noise_o, &e->noise_n, &e->loss_b, &e->logit_b})
    if ((rc = e->alloc(q, B))) return bad(rc);
  const long long B2 = 3LL * B;  // rows of the forward buffers (online s, online s', target s')
  for (float** q : {&e->rstd1, &e->rstd2})
    if ((rc = e->alloc(q, B2))) return bad(rc);
  long long maxact = 0;
  for (int s = 0; s < 3; ++s) {
    Stack& k = e->stk[s];
    const long long big = (long long)B * k.hin * k.hin * k.co, sm = (long long)B * k.ho * k.ho * k.co;
    maxact = std::max({maxact, big, (long long)B * k.hin * k.hin * k.ci});
    if ((rc = e->alloc(&k.conv0, 3 * big)) || (rc = e->alloc(&k.arg, 3 * sm))) return bad(rc);
    for (float** q : {&k.c[0], &k.c[1], &k.c[2], &k.r[0], &k.r[1]})
      if ((rc = e->alloc(q, 3 * sm))) return bad(rc);
  }
  if ((rc = e->alloc(&e->stk[0].xin_own, 3 * img))) return bad(rc);  // augmented [obs | next_obs | next_obs]
  e->nobs = e->stk[0].xin_own + img;
  for (float** q : {&e->ga, &e->gb, &e->gc})
    if ((rc = e->alloc(q, maxact))) return bad(rc);
  for (float** q : {&e->feat, &e->xhat1, &e->ln1})
    if ((rc = e->alloc(q, B2 * F))) return bad(rc);
  for (float** q : {&e->dln1, &e->dfeat})
    if ((rc = e->alloc(q, (long long)B * F))) return bad(rc);
  for (float** q : {&e->z1, &e->xhat2, &e->h2})
    if ((rc = e->alloc(q, B2 * H))) return bad(rc);
  for (float** q : {&e->dh2, &e->dz1})
    if ((rc = e->alloc(q, (long long)B * H))) return bad(rc);
  if ((rc = e->alloc(&e->hc, B2 * NC))) return bad(rc);
  for (float** q : {&e->hc_on, &e->hc_tg, &e->dhc})
    if ((rc = e->alloc(q, (long long)B * NC))) return bad(rc);
  if ((rc = e->alloc(&e->m, (long long)B * Z))) return bad(rc);
  {  // per-conv partial regions and the segment table of the one partial-sum launch
    std::vector<drq::SumSeg> segs;
    long long total = 0;
    for (int s = 0; s < 3; ++s)
      for (int j = 0; j < 5; ++j) {
        const Stack& k = e->stk[s];
        const int hh = j == 0 ? k.hin : k.ho, ci = j == 0 ? k.ci : k.co;
        total += (long long)drq::conv_wgrad_blocks(B, hh, hh, ci, k.co) * (9LL * ci * k.co + k.co);
      }
    float* all = nullptr;
    if ((rc = e->alloc(&all, total))) return bad(rc);
    int blk = 0;
    for (int s = 0; s < 3; ++s)
      for (int j = 0; j < 5; ++j) {
        const Stack& k = e->stk[s];
        const int hh = j == 0 ? k.hin : k.ho, ci = j == 0 ? k.ci : k.co;
        const int G = drq::conv_wgrad_blocks(B, hh, hh, ci, k.co), n = 9 * ci * k.co + k.co;
        e->wparts[s][j] = all;
        segs.push_back({all, e->g + k.cw[j], e->g + k.cb[j], G, n, 9 * ci * k.co, blk});
        blk += drq::sum_parts_blocks(ci, k.co);
        all += (long long)G * n;
      }
    e->seg_blocks = blk;
    if ((rc = e->alloc(&e->d_segs, (long long)segs.size())) ||
        hipMemcpy(e->d_segs, segs.data(), sizeof(drq::SumSeg) * segs.size(), hipMemcpyHostToDevice) != hipSuccess)
      return bad(rc ? rc : fail(-5, "segment table upload"));
  }
  e->ws_floats = std::max({gemm_ws_floats(H, NC, 1, gemm_splits(H, NC, B, 1)),
                           gemm_ws_floats(F, H, 1, gemm_splits(F, H, B, 1)),
                           gemm_ws_floats(B, H, 1, gemm_splits(B, H, F, 1)),
                           gemm_ws_floats(B, NC, 1, gemm_splits(B, NC, H, 1)),
                           gemm_ws_floats(B, H, 1, gemm_splits(B, H, NC, 1)),
                           gemm_ws_floats(B, F, 1, gemm_splits(B, F, H, 1)),
                           gemm_ws_floats(2 * B, H, 1, gemm_splits(2 * B, H, F, 1)),
                           gemm_ws_floats(2 * B, NC, 1, gemm_splits(2 * B, NC, H, 1))});
  if ((rc = e->alloc(&e->ws, e->ws_floats))) return bad(rc);
  if ((rc = e->alloc(&e->part, 2 * 1024)) || (rc = e->alloc(&e->logs, DRQ_NUM_LOGS))) return bad(rc);
  if ((rc = e->alloc(&e->trunc, B))) return bad(rc);
  e->img = (long long)c->in_ch * c->hw * c->hw;
  if (c->capacity > 0) {
    if (c->capacity <= c->nstep + 6 || c->nstep < 1 || e->img % 16 != 0 || c->capacity > (1LL << 30))
      return bad(fail(-22, "buffer: capacity > nstep + 6, frames of 16-B multiples"));
    e->cap = c->capacity;
    e->n_per_task = B / e->T;
    if (c->buffer_kind != DRQ_BUFFER_MEMORY_EFFICIENT && c->buffer_kind != DRQ_BUFFER_ATARI)
      return bad(fail(-22, "buffer_kind"));
    if ((rc = e->alloc(&e->store, e->cap * e->T * e->img))) return bad(rc);
    if (c->buffer_kind == DRQ_BUFFER_ATARI && (rc = e->alloc(&e->nstore, e->cap * e->T * e->img))) return bad(rc);
    if ((rc = e->alloc(&e->b_act, e->cap * e->T))) return bad(rc);
    for (float** q : {&e->b_rew, &e->b_done, &e->b_trunc})
      if ((rc = e->alloc(q, e->cap * e->T))) return bad(rc);
    if ((rc = e->alloc(&e->d_minmax, 2 * e->T)) || (rc = e->alloc(&e->rng, 1)) || (rc = e->alloc(&e->jump, 65 * 4)) ||
        (rc = e->alloc(&e->idx, e->n_per_task)) || (rc = e->alloc(&e->r_slot, (long long)drq_engine::ROWS_STEPS * B)) ||
        (rc = e->alloc(&e->r_task, (long long)drq_engine::ROWS_STEPS * B)))
      return bad(rc);
    unsigned long long jt[65 * 4];
    pcg_jump_table(jt);
    if (hipMemcpy(e->jump, jt, sizeof(jt), hipMemcpyHostToDevice) != hipSuccess) return bad(fail(-5, "jump table"));
    const size_t ring = (size_t)c->nstep * e->T;
    e->ns_obs.assign(ring * e->img, 0);
    e->ns_next.assign(ring * e->img, 0);
    e->ns_act.assign(ring, 0);
    e->ns_rew.assign(ring, 0.f);
    e->ns_trunc.assign(ring, 0.f);
    e->ns_done.assign(ring, 0.f);
    e->minmax.assign(2 * e->T, 0.0);
    for (int t = 0; t < e->T; ++t) {
      e->minmax[t] = INFINITY;
      e->minmax[e->T + t] = -INFINITY;
    }
  }
  if (hipStreamSynchronize(e->st) != hipSuccess) return bad(fail(-5, "init sync"));
  *out = e;
  return 0;
}

void drq_destroy(drq_engine* e) {
  if (!e) return;
  if (e->st) (void)hipStreamSynchronize(e->st);
  for (hipEvent_t x : e->ev) (void)hipEventDestroy(x);
  for (void* q : e->allocs) (void)hipFree(q);
  if (e->st) (void)hipStreamDestroy(e->st);
  delete e;
}

long long drq_num_params(const drq_engine* e) { return e ? e->n_flax : -22; }

static float* which_buf(drq_engine* e, int which) {
  switch (which) {
    case DRQ_PARAMS: return e->p;
    case DRQ_TARGET: return e->tgt;
    case DRQ_ADAM_MU: return e->mu;
    case DRQ_ADAM_NU: return e->nu;
    case DRQ_GRAD: return e->g;
    default: return nullptr;
  }
}

int drq_set_params(drq_engine* e, int which, const float* flat, long long n) {
  if (!e || !flat) return fail(-22, "null argument");
  float* dst = which == DRQ_GRAD ? nullptr : which_buf(e, which);
  if (!dst) return fail(-22, "bad buffer id");
  if (n != e->n_flax) return fail(-22, "parameter count mismatch");
  std::vector<float> host((size_t)e->n_int, 0.f);
  for (const auto& mp : e->map)
    for (long long r = 0; r < mp.rows; ++r)
      std::memcpy(&host[(size_t)(mp.i + r * mp.ld)], flat + mp.f + r * mp.n, sizeof(float) * (size_t)mp.n);
  if (hipMemcpyAsync(dst, host.data(), sizeof(float) * host.size(), hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "upload failed");
  return 0;
}

int drq_get_params(drq_engine* e, int which, float* flat, long long n) {
  if (!e || !flat) return fail(-22, "null argument");
  float* src = which_buf(e, which);
  if (!src) return fail(-22, "bad buffer id");
  if (n != e->n_flax) return fail(-22, "parameter count mismatch");
  std::vector<float> host((size_t)e->n_int);
  if (hipMemcpyAsync(host.data(), src, sizeof(float) * host.size(), hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "download failed");
  for (const auto& mp : e->map)
    for (long long r = 0; r < mp.rows; ++r)
      std::memcpy(flat + mp.f + r * mp.n, &host[(size_t)(mp.i + r * mp.ld)], sizeof(float) * (size_t)mp.n);
  return 0;
}

int drq_set_step(drq_engine* e, int adam_count) {
  if (!e || adam_count < 0) return fail(-22, "bad argument");
  e->count = adam_count;
  return 0;
}

int drq_get_step(drq_engine* e, int* adam_count) {
  if (!e || !adam_count) return fail(-22, "null argument");
  *adam_count = e->count;
  return 0;
}

int drq_update(drq_engine* e, const drq_batch* b) {
  if (!e || !b) return fail(-22, "null argument");
  const int B = e->B;
  const size_t img = (size_t)B * e->cfg.in_ch * e->cfg.hw * e->cfg.hw;
  int rc;
  if ((rc = copy_in(e->obs_u8, b->obs, img, e->st)) || (rc = copy_in(e->nobs_u8, b->next_obs, img, e->st)) ||
      (rc = copy_in(e->act, b->actions, sizeof(int) * B, e->st)) ||
      (rc = copy_in(e->task, b->task_ids, sizeof(int) * B, e->st)) ||
      (rc = copy_in(e->rew, b->rewards, sizeof(float) * B, e->st)) ||
      (rc = copy_in(e->done, b->dones, sizeof(float) * B, e->st)) ||
      (rc = copy_in(e->crop_o, b->crop_obs, sizeof(int) * 2 * B, e->st)) ||
      (rc = copy_in(e->crop_n, b->crop_next, sizeof(int) * 2 * B, e->st)) ||
      (rc = copy_in(e->noise_o, b->noise_obs, sizeof(float) * B, e->st)) ||
      (rc = copy_in(e->noise_n, b->noise_next, sizeof(float) * B, e->st)))
    return rc;
  e->step();
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_update_resident(drq_engine* e, int steps) {
  if (!e || steps < 0) return fail(-22, "bad argument");
  for (int i = 0; i < steps; ++i) {
    e->draw_aug();
    e->step();
  }
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_q_values(drq_engine* e, const unsigned char* obs, const int* task_ids, const int* crop, const float* noise,
                 int n, float* q) {
  if (!e || !q) return fail(-22, "null argument");
  if (n < 1 || n > e->B) return fail(-22, "n must be in [1, batch]");
  const size_t img = (size_t)n * e->cfg.in_ch * e->cfg.hw * e->cfg.hw;
  int rc;
  if ((rc = copy_in(e->obs_u8, obs, img, e->st)) || (rc = copy_in(e->task, task_ids, sizeof(int) * n, e->st)) ||
      (rc = copy_in(e->crop_o, crop, sizeof(int) * 2 * n, e->st)) ||
      (rc = copy_in(e->noise_o, noise, sizeof(float) * n, e->st)))
    return rc;
  e->q_values(n, e->m);  // m (B x Z floats) as scratch for the n x A values
  if (hipMemcpyAsync(q, e->m, sizeof(float) * (size_t)n * e->A, hipMemcpyDefault, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "q download failed");
  return 0;
}

int drq_buffer_add(drq_engine* e, const unsigned char* obs, const unsigned char* next_obs, const int* action,
                   const float* reward, const float* truncate, const float* done) {
  if (!e || !obs || !next_obs || !action || !reward || !truncate || !done) return fail(-22, "null argument");
  if (!e->store) return fail(-95, "engine created without a buffer (capacity 0)");
  return e->buffer_add(obs, next_obs, action, reward, truncate, done);
}

int drq_buffer_state(drq_engine* e, long long* pos, int* full) {
  if (!e || !pos || !full) return fail(-22, "null argument");
  *pos = e->pos;
  *full = e->full;
  return 0;
}

int drq_rng_set(drq_engine* e, unsigned long long shi, unsigned long long slo, unsigned long long ihi,
                unsigned long long ilo, int has32, unsigned int u) {
  if (!e) return fail(-22, "null argument");
  if (!e->rng) return fail(-95, "engine created without a buffer (capacity 0)");
  PcgDev h{shi, slo, ihi, ilo, has32, u};
  if (hipMemcpyAsync(e->rng, &h, sizeof(h), hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "rng upload failed");
  return 0;
}

int drq_sample(drq_engine* e) {
  if (!e) return fail(-22, "null argument");
  if (!e->store) return fail(-95, "engine created without a buffer (capacity 0)");
  if (!e->full && e->pos == 0) return fail(-22, "empty buffer");
  int rc = e->sample();
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_sample_update(drq_engine* e, int steps) {
  if (!e || steps < 0) return fail(-22, "bad argument");
  if (!e->store) return fail(-95, "engine created without a buffer (capacity 0)");
  if (!e->full && e->pos == 0) return fail(-22, "empty buffer");
  for (int i = 0; i < steps; ++i) {
    int rc = e->sample();
    if (rc) return rc;
    e->draw_aug();
    e->step();
  }
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_sample_rows(drq_engine* e, const long long* slots, const int* task_ids) {
  if (!e || !slots || !task_ids) return fail(-22, "null argument");
  if (!e->store) return fail(-95, "engine created without a buffer (capacity 0)");
  int rc;
  if ((rc = e->upload_rows(slots, task_ids, 1)) || (rc = e->sample_rows(e->r_slot, e->r_task))) return rc;
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_sample_rows_update(drq_engine* e, const long long* slots, const int* task_ids, int steps) {
  if (!e || !slots || !task_ids || steps < 0) return fail(-22, "bad argument");
  if (!e->store) return fail(-95, "engine created without a buffer (capacity 0)");
  const long long B = e->B;
  for (int s0 = 0; s0 < steps; s0 += drq_engine::ROWS_STEPS) {
    const int k = std::min(steps - s0, drq_engine::ROWS_STEPS);
    int rc = e->upload_rows(slots + s0 * B, task_ids + s0 * B, k);
    if (rc) return rc;
    for (int i = 0; i < k; ++i) {
      if ((rc = e->sample_rows(e->r_slot + i * B, e->r_task + i * B))) return rc;
      e->draw_aug();
      e->step();
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_rng_get(drq_engine* e, unsigned long long* out6) {
  if (!e || !out6) return fail(-22, "null argument");
  if (!e->rng) return fail(-95, "engine created without a buffer (capacity 0)");
  PcgDev h{};
  if (hipMemcpyAsync(&h, e->rng, sizeof(h), hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "rng download failed");
  out6[0] = h.state_hi;
  out6[1] = h.state_lo;
  out6[2] = h.inc_hi;
  out6[3] = h.inc_lo;
  out6[4] = (unsigned long long)h.has_uint32;
  out6[5] = h.uinteger;
  return 0;
}

int drq_seed_augment(drq_engine* e, unsigned long long seed) {
  if (!e) return fail(-22, "null argument");
  e->aug_seed = seed;
  e->aug_ctr = 0;
  return 0;
}

int drq_read_batch(drq_engine* e, unsigned char* obs, unsigned char* next_obs, int* actions, float* rewards,
                   float* dones, float* truncations, int* task_ids) {
  if (!e) return fail(-22, "null argument");
  const int B = e->B;
  const size_t img = (size_t)B * e->img;
  struct {
    void* dst;
    const void* src;
    size_t n;
  } cp[7] = {{obs, e->obs_u8, img},
             {next_obs, e->nobs_u8, img},
             {actions, e->act, sizeof(int) * B},
             {rewards, e->rew, sizeof(float) * B},
             {dones, e->done, sizeof(float) * B},
             {truncations, e->trunc, sizeof(float) * B},
             {task_ids, e->task, sizeof(int) * B}};
  for (auto& c : cp)
    if (c.dst && hipMemcpyAsync(c.dst, c.src, c.n, hipMemcpyDeviceToHost, e->st) != hipSuccess)
      return fail(-5, "batch download failed");
  return hipStreamSynchronize(e->st) == hipSuccess ? 0 : fail(-5, "stream sync failed");
}

int drq_get_logs(drq_engine* e, float* out) {
  if (!e || !out) return fail(-22, "null argument");
  if (hipMemcpyAsync(out, e->logs, sizeof(float) * DRQ_NUM_LOGS, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "log download failed");
  return 0;
}

int drq_synchronize(drq_engine* e) {
  if (!e) return fail(-22, "null argument");
  return hipStreamSynchronize(e->st) == hipSuccess ? 0 : fail(-5, "stream sync failed");
}

int drq_task_gradient(drq_engine* e, const drq_batch* b, int slot, int num_slots) {
  if (!e || !b) return fail(-22, "null argument");
  if (num_slots < 1 || slot < 0 || slot >= num_slots) return fail(-22, "slot out of range");
  const int B = e->B;
  const size_t img = (size_t)B * e->cfg.in_ch * e->cfg.hw * e->cfg.hw;
  int rc;
  long long have = (long long)e->tg_slots * e->n_flax;
  if ((rc = e->realloc_buf(&e->tg, have, (long long)num_slots * e->n_flax))) return rc;
  e->tg_slots = (int)(have / e->n_flax);
  if ((rc = copy_in(e->obs_u8, b->obs, img, e->st)) || (rc = copy_in(e->nobs_u8, b->next_obs, img, e->st)) ||
      (rc = copy_in(e->act, b->actions, sizeof(int) * B, e->st)) ||
      (rc = copy_in(e->task, b->task_ids, sizeof(int) * B, e->st)) ||
      (rc = copy_in(e->rew, b->rewards, sizeof(float) * B, e->st)) ||
      (rc = copy_in(e->done, b->dones, sizeof(float) * B, e->st)) ||
      (rc = copy_in(e->crop_o, b->crop_obs, sizeof(int) * 2 * B, e->st)) ||
      (rc = copy_in(e->crop_n, b->crop_next, sizeof(int) * 2 * B, e->st)) ||
      (rc = copy_in(e->noise_o, b->noise_obs, sizeof(float) * B, e->st)) ||
      (rc = copy_in(e->noise_n, b->noise_next, sizeof(float) * B, e->st)))
    return rc;
  e->grad_pass();
  drq::flax_gather(e->g, e->d_map, (int)e->map.size(), e->map_max, e->tg + (long long)slot * e->n_flax, e->st);
  return hipGetLastError() == hipSuccess ? 0 : fail(-5, "kernel launch failed");
}

int drq_get_task_gradient(drq_engine* e, int slot, float* flat, long long n) {
  if (!e || !flat) return fail(-22, "null argument");
  if (slot < 0 || slot >= e->tg_slots) return fail(-22, "slot out of range");
  if (n != e->n_flax) return fail(-22, "parameter count mismatch");
  if (hipMemcpyAsync(flat, e->tg + (long long)slot * e->n_flax, sizeof(float) * n, hipMemcpyDefault, e->st) !=
          hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "download failed");
  return 0;
}

int drq_project_task_gradients(drq_engine* e, int num_slots, int proj_dim, long long chunk, int seed, float* out) {
  if (!e || !out) return fail(-22, "null argument");
  if (num_slots < 1 || num_slots > e->tg_slots) return fail(-22, "num_slots exceeds the stored task gradients");
  if (proj_dim < 1 || chunk < 1) return fail(-22, "proj_dim and chunk must be positive");
  const long long P = e->n_flax;
  int rc;
  if ((rc = e->realloc_buf(&e->jl_part, e->jl_part_n, drq::jl_part_floats(P, proj_dim))) ||
      (rc = e->realloc_buf(&e->jl_out, e->jl_out_n, (long long)num_slots * proj_dim)))
    return rc;
  const int TM = drq::jl_max_tasks();
  for (int t0 = 0; t0 < num_slots; t0 += TM)
    drq::jl_project(e->tg + (long long)t0 * P, P, std::min(TM, num_slots - t0), P, proj_dim, chunk, seed, e->jl_part,
                    e->jl_out + (long long)t0 * proj_dim, proj_dim, e->st);
  if (hipGetLastError() != hipSuccess) return fail(-5, "kernel launch failed");
  if (hipMemcpyAsync(out, e->jl_out, sizeof(float) * (size_t)num_slots * proj_dim, hipMemcpyDefault, e->st) !=
          hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return fail(-5, "download failed");
  return 0;
}

int drq_set_timing(drq_engine* e, int on) {
  if (!e) return fail(-22, "null argument");
  if (hipStreamSynchronize(e->st) != hipSuccess) return fail(-5, "stream sync failed");
  e->timing = on != 0;
  e->ev_used = 0;
  e->t_flops = 0;
  e->t_launches = 0;
  return 0;
}

int drq_timing(drq_engine* e, double* ms, long long* launches, double* flops) {
  if (!e || !ms || !launches || !flops) return fail(-22, "null argument");
  if (hipStreamSynchronize(e->st) != hipSuccess) return fail(-5, "stream sync failed");
  double total = 0;
  for (size_t i = 0; i + 1 < e->ev_used; i += 2) {
    float x = 0;
    if (hipEventElapsedTime(&x, e->ev[i], e->ev[i + 1]) != hipSuccess) return fail(-5, "event timing failed");
    total += x;
  }
  *ms = total;
  *launches = e->t_launches;
  *flops = e->t_flops;
  return 0;
}

}  // extern "C"
