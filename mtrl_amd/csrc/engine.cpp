// engine.cpp -- the MTSAC update engine behind include/mtsac.h (C-ABI).
//
// Orchestrates one multi-task SAC gradient step (reference _update_inner,
// mtrl/rl/algorithms/mtsac.py:1173-1247) as a fixed sequence of HIP kernels on one
// stream: device index stream + gather, actor forward on s' (a', logpi'), target
// critic (y), critic forward/backward, clip+Adam+Polyak, actor forward, critic
// forward with the UPDATED critic, critic data-grad into the action columns,
// actor backward, clip+Adam, temperature update.  Every pointer is fixed at
// creation, so the whole step is captured once into a hipGraph and replayed.
//
// Task sharding (multi-GPU): an engine owns tasks [task_begin, task_begin+task_count);
// trunk parameters are replicated, heads are local.  Per network one RCCL
// all-reduce(sum) runs over the contiguous trunk-gradient range plus a small
// scalar tail (local head |g|^2, loss sums, temperature grads), so the global
// clip norm and the logged losses equal the single-device ones.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtsac.h"
#include "../../include/mtsac_debug.h"
#include "kernels.h"

using namespace mtsac;

namespace {

thread_local std::string g_last_error;
int g_bfrag_mode = -1;  // mtsac_debug_set_bfrag: -1 by shape (and MTSAC_BFRAG), 0 off, 1 allowed

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(-5, std::string(#expr) + ": " + hipGetErrorString(_e));                  \
  } while (0)

constexpr int MAXD = 8;
constexpr long long ALIGN = 64;  // floats (256 B)
constexpr int EXTRA = 128;       // scalar tail of each gradient buffer (all-reduced with the trunk)
constexpr int PART = 1024;       // max partial-sum blocks

long long align_up(long long x, long long a) { return (x + a - 1) / a * a; }

struct Net {
  int in_dim = 0, in_ld = 0, width = 0, depth = 0, T_l = 0, hd = 0, E = 1;
  long long off_hb = 0, off_hW = 0, off_b[MAXD] = {}, off_W[MAXD] = {};
  long long ms_hb = 0, ms_hW = 0, ms_b = 0, ms_W[MAXD] = {};  // member strides
  long long n_flat = 0, trunk_off = 0, n_params = 0;
  std::vector<std::pair<long long, long long>> leaves;  // (offset, count) in flax order
  float *p = nullptr, *g = nullptr, *m = nullptr, *v = nullptr, *tgt = nullptr;
  // transposed hidden kernels W_i^T ([E][out][in], i >= 1) of p (wt[0]) and tgt (wt[1]): the
  // trunk forward runs as an NT product against them (k-contiguous operands on both sides)
  float* wt[2][MAXD] = {};
  // split3: bf16 planes of the hidden kernels W_i ([E][3][wrows][wld], i >= 1) of p ([0]) and tgt
  // ([1]), rows and columns rounded up to 32 with zeros.  The forward reads them k-major (its
  // B(n, k) = W[k][n]), the data grad row-major (B(n, k) = W[n][k]).  Activation / data-grad
  // planes of this net are [E][3][arows][ald] (arows = B rounded up to 32 with zero rows,
  // ald = width rounded up to 32).
  __bf16* wp[2][MAXD] = {};
  long long wld = 0, wrows = 0, arows = 0, ald = 0;
  // krows: rows of one batch pass rounded up to 32 (the weight grad's K); arows: rows of the
  // activation planes (= krows, or for the actor, whose forward runs ONCE over [s | s'], krows + B
  // rounded up: the s rows first, the s' rows from row krows)
  long long krows = 0;
  // gemm_x3f path (row-major x row-major, gemm_x3f.hip) for the hidden layers' forward and data
  // grad: W_i^T planes ([E][3][width (out)][ald (in)], i >= 1) of p ([0]) and tgt ([1]); hidden
  // activations then keep planes only (their ReLU mask is read from the high plane)
  bool x3f = false;
  __bf16* wtp[2][MAXD] = {};
  // layer i's GEMM-read weight planes (wtp[.][i], and wp[.][i] for the data grad) in the fragment
  // layout (gemm_common.h frag_off: gemm_x3f's B wave loads read whole lines); set when every GEMM
  // that reads them runs on gemm_x3f (engine frag_probe; no other kernel reads the layout)
  bool bfrag[MAXD] = {};
  // the actor's head kernel transposed per task ([T_l][hd][W], heads.hip HeadParams::WhT): the policy
  // heads' weight loads read whole lines; rewritten with the planes after every write of p
  float* whT = nullptr;
  // column-sum partials of dz[i] written by the pass that produces it (head backward, gemm_x3f data
  // grad): [E][chunks][width]; dbp_chunks[i] > 0 when the current step's dz[i] came with them
  float* dbp[MAXD] = {};
  int dbp_chunks[MAXD] = {};
  // one GPU (no collective reads a layer's gradient before the optimizer): the weight grads' finishes
  // (split-K slab sums, bias grads from column sums) are collected in fin_sink and run in ONE launch at
  // the start of the network's optimizer; ws_wg[i] holds layer i's slabs until then
  float* ws_wg[MAXD] = {};
  FinishSink fin_sink;
  long long wtk(int i) const { return i == 0 ? xld : ald; }  // K (padded in-dim) of layer i
  long long wtps(int i = 1) const { return (long long)width * wtk(i); }
  long long xld = 0;  // input planes' row stride = layer-0 kernel plane rows (in_dim rounded up to 32)
  long long aps() const { return arows * ald; }  // plane stride of activation planes
  long long wps() const { return wrows * wld; }  // plane stride of hidden kernel planes
  long long w0ps() const { return xld * wld; }   // plane stride of the layer-0 kernel planes
  long long kps(int i) const { return i == 0 ? w0ps() : wps(); }
  OptScalars* sc = nullptr;
  // fused optimizer (optimize()): |g|^2 partials of the trunk / heads, |p_new|^2 partials of the
  // heads / trunk and their counts from the last launch (the parameter norms are summed in the tail)
  float *gparts = nullptr, *hparts = nullptr, *pph = nullptr, *ppt = nullptr;
  int n_pph = 0, n_ppt = 0;

  void layout(int in, int in_ld_, int W, int D, int T, int hd_, int E_) {
    in_dim = in; in_ld = in_ld_; width = W; depth = D; T_l = T; hd = hd_; E = E_;
    long long o = 0;
    auto leaf = [&](long long member, long long& off, long long& ms) {
      off = o;
      ms = member;
      leaves.push_back({o, member * E});
      n_params += member * E;
      o = align_up(o + member * E, ALIGN);
    };
    leaf((long long)T * hd, off_hb, ms_hb);
    leaf((long long)T * W * hd, off_hW, ms_hW);
    trunk_off = o;
    int fan = in;
    for (int i = 0; i < D; ++i) {
      leaf(W, off_b[i], ms_b);
      leaf((long long)fan * W, off_W[i], ms_W[i]);
      fan = W;
    }
    n_flat = o;
  }
};

}  // namespace

struct mtsac_engine {
  mtsac_config cfg{};
  int device = 0;
  hipStream_t st = nullptr, s1 = nullptr, s2 = nullptr, s3 = nullptr;
  hipStream_t s4 = nullptr;  // lane 4: the trunk-gradient all-reduce buckets (one collective stream)
  hipStream_t cur = nullptr;
  std::vector<hipEvent_t> evpool;
  size_t ev_next = 0;
  bool ev_rotate = getenv("MTSAC_EV_ROTATE") != nullptr;   // experiments (race hunt)
  bool lanes_alt = getenv("MTSAC_LANES_ALT") != nullptr;   // experiments: every step on the overlap lanes
  int T_l = 0, T_g = 0, A = 0, D = 0, B = 0, n = 0, R = 0, ld_a = 0, ld_c = 0, B_glob = 0;
  Net actor, critic;
  // replay
  float* store = nullptr;
  long long* buf_size = nullptr;  // device: pos or capacity
  long long h_pos = 0;
  int h_full = 0;
  PcgDev* rng = nullptr;
  unsigned long long* jump = nullptr;
  int* idx = nullptr;
  double *rmin = nullptr, *rmax = nullptr;  // per-task reward min / max (device-authoritative)
  // async add: pinned staging ring, each slot reusable once its event (after the H2D copy) fired
  static constexpr int NSTAGE = 32;
  float* stage_h = nullptr;
  hipEvent_t stage_ev[NSTAGE] = {};
  int stage_next = 0;
  hipEvent_t add_ev = nullptr;  // orders device-pointer adds after the legacy default stream
  // device-pointer adds: the caller's arrays are packed into an engine-owned staging record on a side
  // stream (sa) that waits only on the producer; the producer waits only on that pack, and the engine
  // stream copies the record into the store in update order (no collection behind queued updates)
  hipStream_t sa = nullptr;
  float* dstage = nullptr;
  hipEvent_t dstage_ev[NSTAGE] = {}, dpack_ev[NSTAGE] = {};
  int dstage_next = 0;
  // inputs
  // xa holds [s | s'] for the actor's single forward: xan = xa + krows * ld_a
  float *xa = nullptr, *xan = nullptr, *xc = nullptr, *xcn = nullptr, *xcp = nullptr;
  int Ma = 0;  // rows of the actor forward over [s | s'] (krows + B; pad rows are zero inputs)
  // Cross-step pipelining (eager update_many): step k+1's gather and critic(s, a) forward run beside
  // step k's actor backward, trunk all-reduce and Adam.  What the gather writes and step k's tail
  // still reads -- the actor input rows (its layer-0 weight grad) and the task row lists (actor
  // heads, temperature) -- alternates between two sets; everything else the early segments write
  // is dead by the time step k's actor-loss pass (s_ap) has run, which they wait for.
  struct InSet {
    float* xa;
    __bf16* xap;  // planes of xa (the input-layer GEMMs' operand; the weight grad reads them after s_ap)
    int *task, *counts, *rows;
  };
  InSet inset[2] = {};
  int inset_cur = 0;
  // Device-sampled batches are interleaved (row i*T_l + t, buffers.py:548), so their per-task row
  // lists are fixed: counts = n, rows[t][i] = i*T_l + t, uploaded once (no task_rows launch per step)
  int *s_counts = nullptr, *s_rows = nullptr;
  hipEvent_t ev_ap[2] = {}, ev_tail[2] = {};  // step k's s_ap / last segment, by step parity
  bool have_prev = false;                      // a pipelined step k is in flight (its events valid)
  // Cross-step pipelining of eager update_many: -1 auto (on when the trunk gradients go through a
  // device collective -- RCCL or the modelled one -- where it hides the actor's all-reduce and Adam),
  // 0 off, 1 on.  MTSAC_PIPELINE / mtsac_debug_set_pipeline override.
  int pipeline_req = [] {
    if (getenv("MTSAC_NO_PIPELINE")) return 0;
    const char* v = getenv("MTSAC_PIPELINE");
    return v ? atoi(v) : -1;
  }();
  // one-stream pipelined issue: the next step's gather + critic(s, a) forward go to the prefetch
  // stream (s2) while the previous step's tail runs on the main stream
  bool pf_issue = false;
  // modelled collective (mtsac_debug_set_collective_model): a one-GPU run issues, at the RCCL points
  // and on the collective stream, a delay of what the all-reduce of each bucket costs on nranks GPUs
  struct CollModel {
    int nranks = 1;
    double gbps = 0.0;
    int blocks = 8;
    bool poison = false;
  } cmodel;
  float* cm_shadow = nullptr;
  long long cm_cap = 0;
  bool dev_collective() const { return comm != nullptr || cmodel.nranks > 1; }
  bool pipeline_on() const { return pipeline_req > 0 || (pipeline_req < 0 && dev_collective()); }
  int step_par = 0;
  float *rew = nullptr, *done = nullptr, *tw = nullptr;
  int* task = nullptr;
  int *counts = nullptr, *rows = nullptr;
  // user-batch staging
  float *u_obs = nullptr, *u_act = nullptr, *u_nobs = nullptr, *u_done = nullptr, *u_rew = nullptr;
  float *eps_n = nullptr, *eps_c = nullptr;
  // activations / grads
  float* ha[MAXD] = {};   // actor activations over [s | s'] (rows [0, B) and [krows, krows + B))
  float* han[MAXD] = {};  // = ha[i] + krows * width: the s' rows
  float* hc[MAXD] = {};
  float* hct[MAXD] = {};  // target-critic activations (concurrent with hc)
  float* dza[MAXD] = {};  // per-layer pre-activation grads
  float* dzc[MAXD] = {};
  // split3 planes of the GEMM operands among them (layers 0..D-2 of activations, 1..D-1 of grads)
  bool planes = false;
  // the input layer's weight grad on k-major planes (gemm_x3p; dz[0] planes + bias partials from the
  // data-grad epilogue) instead of the on-the-fly split kernel: split2h always, split3 below 4096 rows
  // (measured, profiles/r3ff_input_wgrad_ab.txt: MT10/W400 +1.5 %, MT50/W2048 split3 at 6400 rows
  // -0.5 %; split2h S3 -54 us per step, profiles/r5n_step_ab.txt); MTSAC_INPUT_WGRAD=0 / 1 forces
  // either form (set at create)
  bool in_wgrad_planes = false;
  int np = 3;  // operand planes the plane GEMMs read: 3 (split3), 1 (bf16) or 2 (split2h: fp16)
  // ---- precision split2h: a device record (kernels.h PlaneRec: exponent + partial maxima) per fp16
  // plane tensor; n = the partial maxima its last producer wrote (0: consumers bound it by 2^(15 - e))
  bool h2 = false;
  struct RecRef {
    PlaneRec* d = nullptr;
    int n = 0;
  };
  PlaneRec* recs = nullptr;
  RecRef r_in[2];         // the step's input planes (xa / xc / xc_next / xc_pi), per input set
  RecRef r_w[2][2];       // weights [0 actor, 1 critic][0 params, 1 Polyak target]
  RecRef r_ac[3][MAXD];   // activation planes: actor (hap), critic (hcp), target critic (hctp)
  RecRef r_dz[2][MAXD];   // data-grad planes: actor (dzap), critic (dzcp)
  RecRef r_dq, r_dout;    // the head backwards' inputs: critic dq, actor dout (partial maxima only)
  float* bufmax = nullptr;  // max |stored obs / action / next_obs| (the input planes' bound)
  float* ubmax = nullptr;   // the same over a user batch
  float* wparts[2] = {};    // the optimizer's per-block max |p_new| [actor, critic] and the target's
  float* tparts = nullptr;
  int wgrid[2] = {}, wbh[2] = {};  // the last optimizer launch's grid and head blocks per network
  RecRef* act_rec(__bf16** actp) {
    return actp == hap || actp == hap_s2 ? r_ac[0] : actp == hcp ? r_ac[1] : actp == hctp ? r_ac[2] : nullptr;
  }
  RecRef* dz_rec(__bf16** dzp) { return dzp == dzap ? r_dz[0] : dzp == dzcp ? r_dz[1] : nullptr; }
  RecRef& w_rec(const Net& net, int which) { return r_w[&net == &critic ? 1 : 0][which]; }
  // |one Adam step| / lr: by Cauchy-Schwarz |m_t| <= (1 - b1) / sqrt((1 - b2)(1 - b1^2 / b2)) sqrt(v_t) for
  // any gradient sequence, times the bias corrections' ratio sqrt(1 - b2^t) / (1 - b1^t) at its worst
  // step t (<= 1 at b1 = 0.9, b2 = 0.999: 7.27 in all); 25 % margin.  Computed once at create.
  float adam_bound = 0.f;
  float adam_step_bound() const { return adam_bound; }
  static float adam_step_bound_of(double b1, double b2) {
    double r = 1.0;
    for (int t = 1; t <= 200000; t = t < 1000 ? t + 1 : t + t / 100) {
      const double f = std::sqrt(1.0 - std::pow(b2, t)) / (1.0 - std::pow(b1, t));
      r = std::max(r, f);
    }
    return (float)(1.25 * r * (1.0 - b1) / std::sqrt((1.0 - b2) * (1.0 - b1 * b1 / b2)));
  }
  // the bound inputs of a split2h plane GEMM: A, B (weights: their planes' range), output C
  void h2_gemm(SplitGemmParams& g, RecRef* a, RecRef* b, RecRef* c, float kmul, bool bias_in_b) {
    if (!h2) return;
    g.ra = a->d;
    g.na = a->n;
    g.rb = b->d;
    g.nb = b->n;
    g.rc = c ? c->d : nullptr;
    g.nparts = c ? &c->n : nullptr;
    if (c) c->n = 0;  // set by the launcher
    g.kmul = kmul;
    g.bias_in_b = bias_in_b ? 1 : 0;
  }
  __bf16* hap[MAXD] = {};
  __bf16* hap_s2[MAXD] = {};  // = hap[i] + krows * ald: the s' rows of the actor's hidden planes
  __bf16* hcp[MAXD] = {};
  __bf16* hctp[MAXD] = {};
  __bf16* dzap[MAXD] = {};
  __bf16* dzcp[MAXD] = {};
  float* cs_part = nullptr;  // column-sum partials (bias grads beside the plane weight-grad GEMM)
  // planes of the GEMM-ready trunk inputs (xa, xan, xc, xcn, xcp): [3][arows][xld]
  struct InPlanes {
    const float* x;
    __bf16* p;
  };
  InPlanes inp[5] = {};
  __bf16* in_planes(const float* X) const {
    for (const InPlanes& q : inp)
      if (q.x == X) return q.p;
    if (X == xan && inp[0].p) return inp[0].p + actor.krows * actor.xld;  // the s' rows of xa's planes
    return nullptr;
  }
  // Split actor forward (device collective, eager one stream): the s' rows (a' for the TD target) run
  // before the critic loss as always, the s rows (pi(s) for the actor loss) beside the critic's trunk
  // all-reduce -- the one stretch of the step where nothing else may run (the rest needs the updated
  // critic).  MTSAC_SPLIT_ACTOR=0 / 1 forces either form.
  int split_actor_req = [] {
    const char* v = getenv("MTSAC_SPLIT_ACTOR");
    return v ? atoi(v) : -1;
  }();
  float *logpi_n = nullptr, *logpi = nullptr, *y = nullptr, *dq = nullptr, *row_a = nullptr, *row_b = nullptr,
        *row_c = nullptr, *alpha_w = nullptr, *cache = nullptr, *dout_a = nullptr;
  float* partials = nullptr;
  // split-K workspaces, one per lane: segments on different lanes may run concurrently, the
  // segments of one lane are ordered by the step DAG (see seg())
  float* ws_lane[5] = {};
  int* cnt_lane[5] = {};  // split-K arrival counters per lane (zero between launches)
  // the in-launch split-K finish (gemm_x3f / gemm_x3p FIN) is opt-in (MTSAC_SPLITK_FIN=1): at the
  // task-shard shapes its 128-256 KB slabs per tile made it slower than the separate finishing pass
  // (profiles/r3t_fin_bench.txt)
  // the in-launch finish (MTSAC_SPLITK_FIN=1; split2h: the two-slice pair hand-off, one slab per tile) is
  // opt-in: on the 7-task shard it measured 1.50 vs 1.43 ms per step against the separate finishing pass
  // (profiles/r5m_*): the finish then runs serially on half the CUs, latency-bound
  int* fin_cnt() {
    static const bool on = [] {
      const char* e = getenv("MTSAC_SPLITK_FIN");
      return e && atoi(e) > 0;
    }();
    return on ? cnt_lane[cur_lane] : nullptr;
  }
  int cur_lane = 0;

  // Net::bfrag[li]: every GEMM that reads layer li's weight planes takes gemm_x3f (no other kernel
  // reads the fragment layout).  The step's parameter sets (trunk_forward's x3f branch, dgrad_layer),
  // probed with placeholder pointers after the workspaces exist; a mismatch with the step surfaces
  // as gemmp's error, never as a silent fallback.
  bool frag_probe(const Net& net, int li) {
    static float f_;
    static __bf16 h_;
    float* F = &f_;
    __bf16* H = &h_;
    const bool is_actor = &net == &actor;
    auto base = [&](int M, long long K, long long ldb) {
      SplitGemmParams g{};
      g.np = np;
      g.lda = K;
      g.ldb = ldb;
      g.M = M;
      g.N = net.width;
      g.K = (int)K;
      g.splits = -1;
      g.ws = ws_lane[0];
      g.cnt = fin_cnt();
      g.b_frag = 1;
      return g;
    };
    std::vector<int> fwd_rows = {B};
    if (is_actor) fwd_rows.push_back((int)(net.krows + B));  // the merged [s | s'] forward
    for (int M : fwd_rows)
      for (int i = li; i == li; ++i) {
        SplitGemmParams g = base(M, net.wtk(i), net.wtk(i));
        g.bias = F;
        if (i == net.depth - 1) {
          g.C = F;
          g.ldc = net.width;
        } else {
          g.Cp = H;
          g.ldcp = net.ald;
        }
        if (!gemm_x3f_ok(g, EPI_BIAS_RELU, net.E)) return false;
      }
    for (int want_db = 0; want_db < 2; ++want_db)
      for (int i = li; i == li && i > 0; ++i) {
        SplitGemmParams g = base(B, net.ald, net.wld);
        g.C = F;
        g.ldc = net.width;
        g.mask16 = H;
        g.ldm = (int)net.ald;
        if (i - 1 >= 1 || want_db) {
          g.Cp = H;
          g.ldcp = net.ald;
        }
        bool ok = false;
        if (g.Cp && want_db) {
          SplitGemmParams q = g;
          q.C = nullptr;
          q.dbp = F;
          ok = gemm_x3f_ok(q, EPI_RELU_MASK, net.E);
        } else if (g.Cp) {
          g.C = nullptr;
        }
        if (!ok && !gemm_x3f_ok(g, EPI_RELU_MASK, net.E)) return false;
      }
    return true;
  }
  float* pn = nullptr;  // [critic trunk |p|^2, actor trunk, critic heads, actor heads]
  float* log_alpha = nullptr;
  float *la_m = nullptr, *la_v = nullptr;
  float* alpha_tmp = nullptr;  // per-task temperature-loss terms (alpha_grad)
  OptScalars* sc_alpha = nullptr;
  float* logs = nullptr;
  unsigned long long* counter = nullptr;
  int* err = nullptr;
  // rollout
  int roll_max = 0;
  float *r_obs = nullptr, *r_x = nullptr, *r_eps = nullptr, *r_act = nullptr, *r_lp = nullptr, *r_dummy = nullptr;
  float* r_h[MAXD] = {};
  int* r_task = nullptr;
  // graph
  bool use_graph = true;
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  bool graph_timed = false;
  // comm
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  mtsac_allreduce_fn hook = nullptr;
  void* hook_user = nullptr;
  // collective hook with the sharded optimizer's ops (mtsac_set_collective_hook)
  mtsac_collective_fn chook = nullptr;
  void* chook_user = nullptr;
  int hook_rank = 0, hook_world = 1;
  // sharded trunk optimizer (ZeRO-1 style, optimize_zero): requested / in force for this step [actor, critic]
  int zero_req = [] {
    const char* v = getenv("MTSAC_ZERO");
    return v ? atoi(v) : 0;
  }();
  bool zstep[2] = {false, false};
  float* zparts = nullptr;  // shard |g|^2 partials
  float* zscr = nullptr;    // the shard Adam launch's |p|^2 partials (the refresh launch's are the ones used)
  std::string comm_error;
  // timing
  bool timing = false;
  bool timing_serial = false;  // timing with every segment on the main stream (solo kernels)
  // Default: every compute segment on the main stream, the RCCL buckets on their own (lane 4), no
  // cross-step overlap.  The 5-lane form (MTSAC_LANES=1, experiments) ran the independent chains of
  // a step on separate streams with event edges, but its results were not bitwise reproducible run
  // to run (last-bit to 7e-5 differences in the logged losses / norms of MT10/W400 in 3 of 8 fresh
  // processes, profiles/r3g_hw_queue_flake.txt; root cause not found in the DAG; fewer hardware
  // queues than streams made it worse) and it was not faster where it could be (MT10/W400: 1194
  // steps/s with lanes, 1265 on one stream, profiles/r3h_bench_c1_*.json).  Lanes are also refused when the
  // process's hardware queues (as started) cannot give every live engine's 5 streams + 3 their own.
  bool one_stream = false;
  bool counted_lanes = false;
  struct TimedLaunch {
    int family;
    double flops;
    int M, N, K, batch;
    hipEvent_t a, b;
  };
  std::vector<TimedLaunch> tl;
  size_t tl_next = 0;
  std::vector<void*> allocs;
  float* dbg_snap[2] = {};  // mtsac_debug_snapshot: ha[top] after the actor forward (0) and after the actor-loss pass (1)
  bool snap_on = false;     // the steps copy into dbg_snap (the buffers stay allocated while off)
  float* dbg_hw = nullptr;  // mtsac_debug_head_selfcheck's scratch head gradient
  // the gemm_x3p geometry (mtsac_debug_x3p_geo) the split-K workspaces (ws_lane, ws_wg) were sized for:
  // a later change could need more slab space than they hold, so the step entry points refuse it
  int geo_at_create = -1;
  int geo_guard() const {
    if (g_x3p_geo == geo_at_create) return 0;
    return fail(-16, "the gemm_x3p geometry changed after this engine was created (mtsac_debug_x3p_geo " +
                         std::to_string(geo_at_create) + " -> " + std::to_string(g_x3p_geo) +
                         "): its split-K workspaces were sized for the old one; restore it or create a new engine");
  }

  ~mtsac_engine() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    for (auto& t : tl) {
      (void)hipEventDestroy(t.a);
      (void)hipEventDestroy(t.b);
    }
    if (comm) {  // finalize first (flushes outstanding work), polling a non-blocking communicator
      ncclResult_t r = ncclCommFinalize(comm);
      for (int i = 0; r == ncclInProgress && i < 200000; ++i) {
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) break;
      }
      ncclCommDestroy(comm);
    }
    for (void* p : allocs) (void)hipFree(p);
    if (stage_h) (void)hipHostFree(stage_h);
    for (hipEvent_t x : stage_ev)
      if (x) (void)hipEventDestroy(x);
    if (add_ev) (void)hipEventDestroy(add_ev);
    for (int k = 0; k < NSTAGE; ++k)
      for (hipEvent_t x : {dstage_ev[k], dpack_ev[k]})
        if (x) (void)hipEventDestroy(x);
    for (hipEvent_t x : {ev_ap[0], ev_ap[1], ev_tail[0], ev_tail[1]})
      if (x) (void)hipEventDestroy(x);
    for (hipEvent_t e : evpool) (void)hipEventDestroy(e);
    for (hipStream_t x : {st, s1, s2, s3, s4, sa})
      if (x) (void)hipStreamDestroy(x);
    if (counted_lanes) {
      Registry& r = registry();
      std::lock_guard<std::mutex> g(r.mu);
      r.live.erase(std::remove(r.live.begin(), r.live.end(), this), r.live.end());
      relane(r);
    }
  }

  static constexpr int LANES = 5;  // st, s1 .. s4
  struct Registry {
    std::mutex mu;
    std::vector<mtsac_engine*> live;
  };
  static Registry& registry() {
    static Registry r;
    return r;
  }
  // Lanes (only when MTSAC_LANES=1) while every live engine's streams, plus a reserve of 3 for the
  // null stream, torch's and RCCL's, fit GPU_MAX_HW_QUEUES (HIP's default 4 when unset; the value
  // the process started with).  Re-decided for ALL live engines whenever one is created or
  // destroyed -- between calls, when every lane has joined the main stream (the last step of
  // update_many joins) -- so in-process multi-engine runs use one stream each.
  // GPU_MAX_HW_QUEUES as the process STARTED (/proc/self/environ): the HIP runtime reads it once,
  // and a value set later from inside the process may or may not have reached it
  static int start_hw_queues() {
    static const int v = [] {
      int q = 4;  // HIP's default
      if (FILE* f = fopen("/proc/self/environ", "rb")) {
        std::string env;
        char buf[4096];
        size_t n;
        while ((n = fread(buf, 1, sizeof(buf), f)) > 0) env.append(buf, n);
        fclose(f);
        const std::string key = "GPU_MAX_HW_QUEUES=";
        for (size_t i = 0; i < env.size();) {
          const size_t e = env.find('\0', i);
          const std::string kv = env.substr(i, (e == std::string::npos ? env.size() : e) - i);
          if (kv.compare(0, key.size(), key) == 0 && atoi(kv.c_str() + key.size()) > 0) q = atoi(kv.c_str() + key.size());
          if (e == std::string::npos) break;
          i = e + 1;
        }
      }
      return q;
    }();
    return v;
  }
  bool force_one = false;  // mtsac_debug_force_one_stream: this engine stays on one stream (not counted)
  static void relane(Registry& r) {
    const char* want = getenv("MTSAC_LANES");
    const int hwq = start_hw_queues();
    int laned = 0;
    for (mtsac_engine* e : r.live) laned += e->force_one ? 0 : 1;
    const bool one = !(want && atoi(want) != 0) || laned * LANES + 3 > hwq;
    for (mtsac_engine* e : r.live) e->one_stream = one || e->force_one || e->s1 == nullptr;  // no lane streams: created without MTSAC_LANES
  }
  void lane_mode_for() {
    Registry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    r.live.push_back(this);
    counted_lanes = true;
    relane(r);
  }

  // Guard zones (debug, MTSAC_GUARD_BYTES=n): every allocation gets n bytes of 0xFF (a NaN in fp32,
  // bf16 and fp16 alike) before and after it; mtsac_debug_check_guards reports any guard a kernel wrote
  // (an out-of-bounds store) -- and an out-of-bounds load inside a guard reads NaN, which the parity
  // tests see.  Off by default (0 bytes).
  struct Guard {
    char* base;
    size_t bytes;
    int line;
  };
  std::vector<Guard> guards;
  static size_t guard_bytes() {
    static const size_t g = [] {
      const char* e = getenv("MTSAC_GUARD_BYTES");
      const long long v = e ? atoll(e) : 0;
      return v > 0 ? (size_t)(v + 255) / 256 * 256 : (size_t)0;
    }();
    return g;
  }

  template <typename T>
  int alloc(T** p, size_t count, int line = __builtin_LINE()) {
    void* q = nullptr;
    size_t bytes = std::max<size_t>(count * sizeof(T), 256);
    bytes = (bytes + 255) / 256 * 256;
    const size_t G = guard_bytes();
    hipError_t e = hipMalloc(&q, bytes + 2 * G);
    if (e != hipSuccess) return fail(-12, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    char* b = reinterpret_cast<char*>(q);
    e = hipMemset(b + G, 0, bytes);
    if (e == hipSuccess && G) e = hipMemset(b, 0xFF, G);
    if (e == hipSuccess && G) e = hipMemset(b + G + bytes, 0xFF, G);
    if (e != hipSuccess) return fail(-5, std::string("hipMemset failed: ") + hipGetErrorString(e));
    allocs.push_back(q);
    if (G) guards.push_back(Guard{b, bytes, line});
    *p = reinterpret_cast<T*>(b + G);
    return 0;
  }

  // ------------------------------------------------------------ streams / timing hooks
  // Work is issued on `cur`; fork/join between the engine's streams goes through a pool of
  // timing-free events (captured into the graph as dependencies).
  void dep(hipStream_t from, hipStream_t to) {
    if (from == to) return;
    if (evpool.empty()) {  // pool is pre-created (no event creation inside a capture)
      comm_error = "event pool exhausted";
      return;
    }
    hipEvent_t e = evpool[ev_next++ % evpool.size()];
    static const bool trace = getenv("MTSAC_TRACE") != nullptr;
    if (trace) fprintf(stderr, "[mtsac] dep %zu %p -> %p\n", ev_next, (void*)from, (void*)to), fflush(stderr);
    hipError_t r = hipEventRecord(e, from);
    if (trace) fprintf(stderr, "[mtsac]   record rc=%d\n", (int)r), fflush(stderr);
    if (r == hipSuccess) r = hipStreamWaitEvent(to, e, 0);
    if (trace) fprintf(stderr, "[mtsac]   wait rc=%d\n", (int)r), fflush(stderr);
    if (r != hipSuccess) comm_error = std::string("stream fork/join: ") + hipGetErrorString(r);
  }

  void t_begin(int family, double flops) {
    if (!timing) return;
    if (tl_next >= tl.size()) {
      TimedLaunch x{};
      (void)hipEventCreate(&x.a);
      (void)hipEventCreate(&x.b);
      tl.push_back(x);
    }
    tl[tl_next].family = family;
    tl[tl_next].flops = flops;
    tl[tl_next].M = tl[tl_next].N = tl[tl_next].K = tl[tl_next].batch = 0;
    (void)hipEventRecord(tl[tl_next].a, cur);
  }
  void t_end() {
    if (!timing) return;
    (void)hipEventRecord(tl[tl_next].b, cur);
    ++tl_next;
  }

  // family: enum mtsac_gemm_family (timing only)
  void gemm(const GemmParams& p, GemmKind kind, int epi, int batch, int family) {
    t_begin(family, 2.0 * (double)p.M * p.N * p.K * batch);
    if (timing) {
      tl[tl_next].M = p.M;
      tl[tl_next].N = p.N;
      tl[tl_next].K = p.K;
      tl[tl_next].batch = batch;
    }
    if (planes)  // split3 / bf16: the plain fp32-operand GEMMs (input-layer weight grad) stay fp32-accurate
      gemm_x3(p, kind, epi, batch, cur);
    else
      gemm_f32(p, kind, epi, batch, cur);
    t_end();
  }

  // kernel behind each GEMM family at its last launch (bench / profile labels)
  std::string fam_kernel[8];

  void gemmp(const SplitGemmParams& p, int epi, int batch, int family) {
    t_begin(family, 2.0 * (double)p.M * p.N * p.K * batch);
    if (timing) {
      tl[tl_next].M = p.M;
      tl[tl_next].N = p.N;
      tl[tl_next].K = p.K;
      tl[tl_next].batch = batch;
    }
    if (gemm_x3f_ok(p, epi, batch)) {
      const bool split = gemm_x3f(p, epi, batch, cur) > 1;
      // the rocprof symbol: gemm_x3f_kernel<BM, EPI, C_OUT, P_OUT, MASK16, TAG, NP> (split-K launches
      // run the raw-slab instance <208 or 128, 0, true, false, false, 0, NP> plus a finishing pass)
      const bool tagged = epi == EPI_BIAS_RELU && p.tag == 1 && p.Cp && !p.C;
      fam_kernel[family] = split ? std::string("gemm_x3f_kernel<") +
                                       std::to_string(gemm_x3f_split_bm(p.M, p.N, p.K, batch)) +
                                       ", 0, true, false, false, 0, " +
                                       std::to_string(p.np == 0 ? 3 : p.np) + "> + splitk_epilogue_kernel"
                                 : std::string("gemm_x3f_kernel<") + std::to_string(gemm_x3f_bm(p, batch)) + ", " +
                                       std::to_string(epi) + ", " +
                                       (p.C ? "true" : "false") + ", " + (p.Cp ? "true" : "false") + ", " +
                                       (p.mask16 ? "true" : "false") + ", " + (tagged ? "8" : "0") + ", " +
                                       std::to_string(p.np == 0 ? 3 : p.np) + ">";
    } else if (p.b_frag) {  // only gemm_x3f reads the fragment layout (Net::bfrag promised it takes the shape)
      comm_error = "B planes in the fragment layout and a shape gemm_x3f does not take";
    } else if (gemm_x3s_ok(p, epi, batch)) {
      gemm_x3s(p, epi, batch, cur);
      const bool tagged = epi == EPI_BIAS_RELU && p.tag == 1 && p.Cp && !p.C;
      fam_kernel[family] = std::string("gemm_x3s_kernel<") + std::to_string(gemm_x3s_ti(p.M, p.N, batch)) + ", " +
                           std::to_string(epi) + ", " + (p.C ? "true" : "false") + ", " + (p.Cp ? "true" : "false") +
                           ", " + (p.mask16 ? "true" : "false") + ", " + (tagged ? "8" : "0") + ", " +
                           std::to_string(p.np == 0 ? 3 : p.np) + ">";
    } else if ((epi == EPI_RELU_MASK && !p.mask) || (!p.C && !p.Cp)) {
      // gemm_x3p's direct epilogue reads an fp32 mask and writes through C or Cp: never launch it
      // on operands it cannot address (a null mask pointer faults the device)
      comm_error = "no plane GEMM kernel for this launch (mask16-only ReLU mask or no output)";
    } else {
      gemm_x3p(p, epi, batch, cur);
      fam_kernel[family] = "gemm_x3p_kernel";
    }
    t_end();
  }

  // planes of the top layer's data grad (written by the head backward), when the trunk has
  // hidden layers that read them
  PlaneOut top_planes(Net& net, __bf16** dzp) {
    PlaneOut po{};
    if (planes && net.depth > 1) {
      po.p = dzp[net.depth - 1];
      po.ld = net.ald;
      po.ps = net.aps();
      po.sm = 3 * net.aps();
      if (h2) {  // bound: hd * max|dout| * (max|head weight| + one Adam step)
        RecRef& top = dz_rec(dzp)[net.depth - 1];
        RecRef& d = &net == &critic ? r_dq : r_dout;
        po.rc = top.d;
        top.n = 0;  // no partial maxima: the planes' range bounds dz_top for the next producer
        po.rd = d.d;
        po.nd = d.n;
        po.rw = w_rec(net, 0).d;
        po.w_add = adam_step_bound() * (&net == &critic ? cfg.critic_lr : cfg.actor_lr);
        po.kmul = (float)net.hd;
      }
    }
    return po;
  }

  // head backward into the top layer's data grad.  With planes the GEMMs read only the planes: the
  // fp32 dz is skipped and (want_db) the bias grad's column sums come out of the same pass.
  void head_bwd(Net& net, const HeadParams& hp, const float* dout, long long s_dout, float** dz, __bf16** dzp,
                bool want_db) {
    const int top = net.depth - 1;
    const PlaneOut po = top_planes(net, dzp);
    if (po.p == nullptr) {
      head_backward_data(hp, dout, s_dout, dz[top], counts, rows, B, T_l, cur, po);
      net.dbp_chunks[top] = 0;
      return;
    }
    head_backward_data(hp, dout, s_dout, nullptr, counts, rows, B, T_l, cur, po, want_db ? net.dbp[top] : nullptr);
    if (want_db) net.dbp_chunks[top] = head_backward_chunks(T_l);
  }

  // head_bwd plus the head's weight/bias grad (head_backward_weight) in ONE launch; false: not
  // launched (fp32 dz without planes, or W % 4 != 0), the caller issues the two passes
  bool head_bwd_both(Net& net, const HeadParams& hp, const float* dout, long long s_dout, __bf16** dzp, bool want_db) {
    const int top = net.depth - 1;
    const PlaneOut po = top_planes(net, dzp);
    if (po.p == nullptr) return false;
    float* dbp = want_db ? net.dbp[top] : nullptr;
    if (!head_backward_both(hp, dout, s_dout, nullptr, counts, rows, B, T_l, po, dbp, net.g + net.off_hW,
                            net.g + net.off_hb, cur))
      return false;
    if (want_db) net.dbp_chunks[top] = head_backward_chunks(T_l);
    return true;
  }

  // ------------------------------------------------------------ trunk passes
  // acts[i] = relu(in_i @ W_i + b_i) for every member (batched over the ensemble)
  // which: 0 / 1 = params is Net::p / Net::tgt (their transposed copies or planes are current),
  // -1 = plain NN form.  actp (split3): planes of acts[0..D-2] to produce, or null.
  void trunk_forward(Net& net, const float* params, int which, const float* X, int ldx, float** acts, __bf16** actp,
                     int M) {
    const bool pl = planes && which >= 0 && actp != nullptr;
    // the input's planes were written with its fp32 rows: the gather (observations, logged
    // actions) and the policy head (the a' / a columns of xc_next / xc_pi); rows >= M and columns
    // >= in_dim stay zero
    __bf16* xp = pl ? in_planes(X) : nullptr;
    for (int i = 0; i < net.depth; ++i) {
      const bool last = i == net.depth - 1;
      if (pl && net.x3f && (i > 0 || xp)) {  // on planes, both row-major: in_i . (W_i^T)^T (gemm_x3f)
        SplitGemmParams g{};
        g.np = np;
        g.A = i == 0 ? xp : actp[i - 1];
        g.lda = i == 0 ? net.xld : net.ald;
        g.pA = i == 0 ? net.arows * net.xld : net.aps();
        g.sA = i == 0 ? 0 : 3 * net.aps();  // the input is shared by the ensemble members
        g.B = net.wtp[which][i];
        g.ldb = net.wtk(i);
        g.pB = net.wtps(i);
        g.sB = 3 * net.wtps(i);
        g.b_frag = net.bfrag[i] ? 1 : 0;
        if (last) {  // the heads read fp32
          g.C = acts[i];
          g.ldc = net.width;
          g.sC = (long long)M * net.width;
        } else {  // the next layer and the data grad's ReLU mask read the planes only
          g.Cp = actp[i];
          g.ldcp = net.ald;
          g.pC = net.aps();
          g.sCp = 3 * net.aps();
        }
        g.bias = params + net.off_b[i];
        g.sBias = net.ms_b;
        g.M = M;
        g.N = net.width;
        g.K = (int)net.wtk(i);
        g.tag = i == 0 ? 1 : 0;
        g.splits = -1;  // split-K when the row tiles do not fill the chip (task shards)
        g.ws = ws_lane[cur_lane];
        g.cnt = fin_cnt();
        if (h2) {
          RecRef* ar = act_rec(actp);
          h2_gemm(g, i == 0 ? &r_in[inset_cur] : &ar[i - 1], &w_rec(net, which), last ? nullptr : &ar[i],
                  (float)(i == 0 ? net.in_dim : net.width), true);
        }
        gemmp(g, EPI_BIAS_RELU, net.E, i == 0 ? MTSAC_FAM_INPUT_FORWARD : MTSAC_FAM_FORWARD);
        continue;
      }
      if (pl && (i > 0 || xp)) {  // on planes: input (row-major) . W_i (k-major)
        SplitGemmParams g{};
        g.np = np;
        g.A = i == 0 ? xp : actp[i - 1];
        g.lda = i == 0 ? net.xld : net.ald;
        g.pA = i == 0 ? net.arows * net.xld : net.aps();
        g.sA = i == 0 ? 0 : 3 * net.aps();
        g.B = net.wp[which][i];
        g.ldb = net.wld;
        g.pB = net.kps(i);
        g.sB = 3 * net.kps(i);
        g.b_kmajor = 1;
        g.C = acts[i];
        g.ldc = net.width;
        g.sC = (long long)M * net.width;
        g.bias = params + net.off_b[i];
        g.sBias = net.ms_b;
        if (!last) {
          g.Cp = actp[i];
          g.ldcp = net.ald;
          g.pC = net.aps();
          g.sCp = 3 * net.aps();
        }
        g.M = M;
        g.N = net.width;
        g.K = (int)(i == 0 ? net.xld : net.ald);
        g.tag = i == 0 ? 1 : 0;
        g.splits = -1;
        g.ws = ws_lane[cur_lane];
        g.cnt = fin_cnt();
        if (h2) {
          RecRef* ar = act_rec(actp);
          h2_gemm(g, i == 0 ? &r_in[inset_cur] : &ar[i - 1], &w_rec(net, which), last ? nullptr : &ar[i],
                  (float)(i == 0 ? net.in_dim : net.width), true);
        }
        gemmp(g, EPI_BIAS_RELU, net.E, i == 0 ? MTSAC_FAM_INPUT_FORWARD : MTSAC_FAM_FORWARD);
        continue;
      }
      GemmParams g{};
      g.A = (i == 0) ? X : acts[i - 1];
      g.lda = (i == 0) ? ldx : net.width;
      g.sA = (i == 0) ? 0 : (long long)M * net.width;
      const bool nt = !planes && which >= 0 && i > 0;
      g.B = nt ? net.wt[which][i] : params + net.off_W[i];
      g.ldb = net.width;
      g.sB = net.ms_W[i];
      g.C = acts[i];
      g.ldc = net.width;
      g.sC = (long long)M * net.width;
      g.bias = params + net.off_b[i];
      g.sBias = net.ms_b;
      g.M = M;
      g.N = net.width;
      g.K = (i == 0) ? net.in_dim : net.width;
      if (pl && !last) {
        g.Cp = actp[i];
        g.ldcp = net.ald;
        g.pC = net.aps();
        g.sCp = 3 * net.aps();
      }
      gemm(g, nt ? GEMM_NT : GEMM_NN, EPI_BIAS_RELU, net.E, i == 0 ? MTSAC_FAM_INPUT_FORWARD : MTSAC_FAM_FORWARD);
    }
  }

  // after every write of params: Net::wt[which] (fp32) or the planes wp[which] (split3);
  // fused: the optimizer already wrote them (see optimize())
  // the optimizer writes the transposed head kernel itself (AdamParams::whT) when its leaf is float4-aligned
  // (one predicate for both sides of the hand-off: refresh_wt skips head_transpose exactly when
  // optimize() gives the head pass AdamParams::whT, whose range must lie inside the heads' part)
  bool whT_fused(const Net& net) const {
    const long long n = (long long)T_l * net.width * net.hd;
    return net.whT && net.E == 1 && net.off_hW % 4 == 0 && n % 4 == 0 && net.off_hW + n <= net.trunk_off;
  }
  void refresh_wt(Net& net, const float* params, int which, hipStream_t s, bool fused = false) {
    if (which == 0 && net.whT && net.E == 1 && !(fused && whT_fused(net)))
      head_transpose(params + net.off_hW, T_l, net.width, net.hd, net.whT, s);
    if (fused && tiles_fusable(net)) return;  // the optimizer wrote every plane the GEMMs read
    for (int i = planes ? 0 : 1; i < net.depth; ++i) {
      if (!planes) {
        transpose_f32(params + net.off_W[i], net.ms_W[i], net.wt[which][i], net.ms_W[i], net.width, net.width, net.E,
                      s);
        continue;
      }
      SplitParams sp{};
      sp.x = params + net.off_W[i];
      sp.ldx = net.width;
      sp.sx = net.ms_W[i];
      sp.rows = i == 0 ? net.in_dim : net.width;
      sp.cols = net.width;
      sp.ldo = net.wld;
      sp.po = net.kps(i);
      sp.so = 3 * net.kps(i);
      sp.out_rows = (int)(i == 0 ? net.xld : net.wrows);
      sp.out_cols = (int)net.wld;
      sp.out = net.wp[which][i];
      sp.e2h = h2 ? &w_rec(net, which).d->e : nullptr;  // split2h: the exponent the optimizer / set_params chose
      sp.frag = net.bfrag[i] ? 1 : 0;
      if (!(fused && planes_fusable(net))) split_planes(sp, false, net.E, s);
      if (net.x3f) {  // W_i^T planes for the gemm_x3f forward (zeros past the in-dim)
        SplitParams st{};
        st.x = params + net.off_W[i];
        st.ldx = net.width;
        st.sx = net.ms_W[i];
        st.rows = i == 0 ? net.in_dim : net.width;  // in
        st.cols = net.width;                        // out
        st.out = net.wtp[which][i];
        st.ldo = net.wtk(i);
        st.po = net.wtps(i);
        st.so = 3 * net.wtps(i);
        st.out_rows = net.width;
        st.out_cols = (int)net.wtk(i);
        st.e2h = sp.e2h;
        st.frag = sp.frag;
        split_planes(st, true, net.E, s);
      }
    }
  }

  // Backward through trunk layer i, split so the two halves can run concurrently:
  //   wgrad_layer: dW_i = in_i^T dz[i] (+ db_i fused into the GEMM's m-tile-0 blocks)
  //   dgrad_layer: dz[i-1] = (dz[i] W_i^T) * [acts[i-1] > 0]
  void wgrad_layer(Net& net, const float* X, int ldx, float** acts, __bf16** actp, float** dz, __bf16** dzp, int i,
                   int M) {
    const __bf16* xp = (planes && i == 0) ? in_planes(X) : nullptr;
    if (planes && (i > 0 || xp) && actp && dzp && dzp[i]) {  // TN on k-major planes; bias grad by column sums
      SplitGemmParams g{};
      g.np = np;
      g.A = i == 0 ? xp : actp[i - 1];
      g.lda = i == 0 ? net.xld : net.ald;
      g.pA = i == 0 ? net.arows * net.xld : net.aps();
      g.sA = i == 0 ? 0 : 3 * net.aps();
      g.a_kmajor = 1;
      g.B = dzp[i];
      g.ldb = net.ald;
      g.pB = net.aps();
      g.sB = 3 * net.aps();
      g.b_kmajor = 1;
      g.C = net.g + net.off_W[i];
      g.ldc = net.width;
      g.sC = net.ms_W[i];
      g.M = i == 0 ? net.in_dim : net.width;
      g.N = net.width;
      g.K = (int)net.krows;  // the s rows (dz is zero past B; the actor's s' rows follow at krows)
      g.tag = i == 0 ? 1 : 0;
      g.splits = -1;  // by tile count (gemm_x3p_splits); the lane workspace is sized for it
      g.ws = ws_lane[cur_lane];
      g.cnt = fin_cnt();
      if (defer_finish()) {  // the finish runs at the start of optimize(net); the slabs wait in ws_wg[i]
        g.ws = net.ws_wg[i];  // (null: this weight grad never splits)
        g.cnt = nullptr;
        g.defer = &net.fin_sink;
      }
      if (net.dbp_chunks[i] > 0) {  // dz[i]'s producer left its column sums: gemm_x3p finishes the bias
        g.cs_part = net.dbp[i];     // grad (in its split-K reduce launch when it has one)
        g.cs_chunks = net.dbp_chunks[i];
        g.cs_db = net.g + net.off_b[i];
        g.cs_sdb = net.ms_b;
      }
      if (h2) h2_gemm(g, i == 0 ? &r_in[inset_cur] : &act_rec(actp)[i - 1], &dz_rec(dzp)[i], nullptr, (float)g.K, false);
      gemmp(g, EPI_STORE, net.E, i == 0 ? MTSAC_FAM_INPUT_WEIGHT_GRAD : MTSAC_FAM_WEIGHT_GRAD);
      if (net.dbp_chunks[i] <= 0)
        colsum(dz[i], M, net.width, net.width, (long long)M * net.width, net.E, cs_part, net.g + net.off_b[i],
               net.ms_b, cur);
      return;
    }
    GemmParams g{};
    g.A = (i == 0) ? X : acts[i - 1];  // [K=rows][M=fan_in] storage -> TA
    g.lda = (i == 0) ? ldx : net.width;
    g.sA = (i == 0) ? 0 : (long long)M * net.width;
    g.B = dz[i];
    g.ldb = net.width;
    g.sB = (long long)M * net.width;
    g.C = net.g + net.off_W[i];
    g.ldc = net.width;
    g.sC = net.ms_W[i];
    g.db = net.g + net.off_b[i];
    g.sDb = net.ms_b;
    g.M = (i == 0) ? net.in_dim : net.width;
    g.N = net.width;
    g.K = M;
    g.splits = gemm_splits(g.M, g.N, g.K, net.E);
    g.ws = ws_lane[cur_lane];
    gemm(g, GEMM_TN, EPI_STORE, net.E, i == 0 ? MTSAC_FAM_INPUT_WEIGHT_GRAD : MTSAC_FAM_WEIGHT_GRAD);
  }

  // want_db: the weight grad of layer i - 1 follows (the trunk backward), so dz[i-1]'s bias-grad
  // column sums are wanted; without it (the actor step's pass through the critic) only the data
  // flows on.  Hidden layers on gemm_x3f keep planes only: their bias grad comes from the
  // epilogue's column sums.
  void dgrad_layer(Net& net, const float* params, float** acts, __bf16** actp, float** dz, __bf16** dzp, int i,
                   int M, bool want_db = true) {
    if (planes && dzp) {  // NT on planes: dz[i] . W_i^T, W_i planes read as [N = in][K = out]
      SplitGemmParams g{};
      g.np = np;
      g.A = dzp[i];
      g.lda = net.ald;
      g.pA = net.aps();
      g.sA = 3 * net.aps();
      g.B = net.wp[0][i];
      g.ldb = net.wld;
      g.pB = net.wps();
      g.sB = 3 * net.wps();
      g.b_frag = net.bfrag[i] ? 1 : 0;
      g.C = dz[i - 1];
      g.ldc = net.width;
      g.sC = (long long)M * net.width;
      if (net.x3f) {  // hidden activations keep planes only: h > 0 <=> its bf16 high plane > 0
        g.mask16 = actp[i - 1];
        g.ldm = (int)net.ald;
        g.sMask = 3 * net.aps();
      } else {
        g.mask = acts[i - 1];
        g.ldm = net.width;
        g.sMask = (long long)M * net.width;
      }
      if (dzp[i - 1] && (i - 1 >= 1 || want_db)) {  // dz[0]'s planes feed only its weight grad
        g.Cp = dzp[i - 1];
        g.ldcp = net.ald;
        g.pC = net.aps();
        g.sCp = 3 * net.aps();
      }
      g.M = M;
      g.N = net.width;
      g.K = (int)net.ald;
      g.splits = -1;
      g.ws = ws_lane[cur_lane];
      g.cnt = fin_cnt();
      g.pMask = net.aps();
      if (h2) h2_gemm(g, &dz_rec(dzp)[i], &w_rec(net, 0), g.Cp ? &dz_rec(dzp)[i - 1] : nullptr, (float)net.width, false);
      if (g.Cp) {  // dz[i-1]'s fp32 copy only feeds the bias grad's column sums
        if (!want_db) {
          g.C = nullptr;
        } else {  // one gemm_x3f pass (no split-K) writes the planes and the column sums
          SplitGemmParams q = g;
          q.C = nullptr;
          q.dbp = net.dbp[i - 1];
          // (or gemm_x3s, the same partials over its 16 TI-row tiles)
          const bool fx = gemm_x3f_ok(q, EPI_RELU_MASK, net.E);
          const bool fs = !fx && !gemm_x3f_ok(g, EPI_RELU_MASK, net.E) && gemm_x3s_ok(q, EPI_RELU_MASK, net.E);
          if (fx || fs) g = q;
          const int bm = fx ? gemm_x3f_out_bm(q, EPI_RELU_MASK, net.E) : 16 * gemm_x3s_ti(M, net.width, net.E);
          net.dbp_chunks[i - 1] = (fx || fs) ? (M + bm - 1) / bm : 0;
        }
      }
      gemmp(g, EPI_RELU_MASK, net.E, MTSAC_FAM_DATA_GRAD);
      return;
    }
    GemmParams g{};
    g.A = dz[i];
    g.lda = net.width;
    g.sA = (long long)M * net.width;
    g.B = params + net.off_W[i];  // W_i (fan_in x W) == [N=fan_in][K=W]
    g.ldb = net.width;
    g.sB = net.ms_W[i];
    g.C = dz[i - 1];
    g.ldc = net.width;
    g.sC = (long long)M * net.width;
    g.mask = acts[i - 1];
    g.ldm = net.width;
    g.sMask = (long long)M * net.width;
    g.M = M;
    g.N = net.width;
    g.K = net.width;
    gemm(g, GEMM_NT, EPI_RELU_MASK, net.E, MTSAC_FAM_DATA_GRAD);
  }

  HeadParams head(Net& net, const float* params, const float* h, int M, const int* tsk) {
    HeadParams hp{};
    hp.h = h;
    hp.Wh = params + net.off_hW;
    hp.WhT = params == net.p ? net.whT : nullptr;
    hp.bh = params + net.off_hb;
    hp.task = tsk;
    hp.B = M;
    hp.W = net.width;
    hp.hd = net.hd;
    hp.E = net.E;
    hp.sWh = net.ms_hW;
    hp.sbh = net.ms_hb;
    hp.sh = (long long)M * net.width;
    hp.fault = reinterpret_cast<unsigned*>(err + 1);  // err[1]: the head backward self-check word (check_err)
    return hp;
  }

  void allreduce(float* buf, size_t count) { coll(0, buf, count); }

  // op 0: all-reduce (sum); 1: reduce-scatter in place (this rank's shard of buf holds the sum);
  // 2: all-gather in place (every rank's shard from its owner).  On the current stream.
  void coll(int op, float* buf, size_t count) {
    if (comm == nullptr && cmodel.nranks > 1) {  // one GPU: the link time of the op, the data as they are
      coll_model_allreduce(buf, (long long)count, cmodel.nranks, cmodel.gbps, cmodel.blocks,
                           cmodel.poison ? cm_shadow : nullptr, cur, op == 0 ? 1.0 : 0.5);
      return;
    }
    if (comm != nullptr) {
      const size_t sh = count / (size_t)nranks;
      ncclResult_t r = op == 0   ? ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm, cur)
                       : op == 1 ? ncclReduceScatter(buf, buf + (size_t)rank * sh, sh, ncclFloat32, ncclSum, comm, cur)
                                 : ncclAllGather(buf + (size_t)rank * sh, buf, sh, ncclFloat32, comm, cur);
      while (r == ncclInProgress) {  // non-blocking communicator: the enqueue completes asynchronously
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) break;
      }
      if (r != ncclSuccess) comm_error = std::string("RCCL collective ") + std::to_string(op) + ": " + ncclGetErrorString(r);
      return;
    }
    if (chook || hook) {
      if (hipStreamSynchronize(cur) != hipSuccess) {
        comm_error = "stream sync before the collective hook failed";
        return;
      }
      if (chook) {
        if (chook(chook_user, op, buf, (int64_t)count) != 0) comm_error = "collective hook failed";
      } else if (op != 0) {
        comm_error = "an all-reduce hook cannot reduce-scatter / all-gather";
      } else if (hook(hook_user, buf, (int64_t)count) != 0) {
        comm_error = "all-reduce hook failed";
      }
    }
  }

  bool sharded() const { return comm != nullptr || hook != nullptr || chook != nullptr || cmodel.nranks > 1; }
  int coll_world() const { return comm ? nranks : cmodel.nranks > 1 ? cmodel.nranks : chook ? hook_world : 1; }
  int coll_rank() const { return comm ? rank : chook ? hook_rank : 0; }

  // the trunk's all-reduce buckets of a network in issue order: hidden layers top-down (b_i, W_i), then
  // layer 0 (b_0, W_0); the whole trunk for a one-layer net
  int zero_buckets(const Net& net, long long* b, long long* e) const {
    int k = 0;
    if (net.depth <= 1) {
      b[0] = net.trunk_off;
      e[0] = net.n_flat;
      return 1;
    }
    for (int i = net.depth - 1; i >= 1; --i) {
      b[k] = net.off_b[i];
      e[k++] = (i + 1 < net.depth) ? net.off_b[i + 1] : net.n_flat;
    }
    b[k] = net.trunk_off;
    e[k++] = net.off_b[1];
    return k;
  }
  // the sharded optimizer applies: requested, a device collective or a collective hook with world > 1,
  // and world divides every bucket into whole float4s
  bool zero_ok(const Net& net) const {
    const int W = coll_world();
    // not under the modelled collective: its reduce-scatter / all-gather move no data, so Adam would
    // update shard 0 of every bucket only (timing runs of the sharded optimizer need real ranks)
    if (zero_req <= 0 || W <= 1 || !(comm || chook) || zparts == nullptr) return false;
    long long b[MAXD + 1], e[MAXD + 1];
    const int n = zero_buckets(net, b, e);
    // optimize_zero skips the gaps around this rank's n shards: up to n + 1 ranges in AdamParams::skip_b/_e
    if (n + 1 > MAX_PLANE_SEGS) return false;
    for (int i = 0; i < n; ++i)
      if ((e[i] - b[i]) % (4LL * W) != 0) return false;
    return true;
  }
  bool zero_of(const Net& net) const { return zstep[&net == &critic ? 1 : 0]; }

  // clip + Adam (+ Polyak) over one network; gradient already complete (and reduced).  Two launches
  // (optim.hip sumsq2 + adam_fused): the |g|^2 partials (and the Adam count), then one update pass
  // over heads, trunk leaves and trunk kernel tiles in which every block recomputes the global norm.
  // The trunk's partials never mix with the heads' (bitwise-identical replicated trunks and norms
  // on every rank); sharded, the heads' |g|^2 is the all-reduced scalar head_sq() left in the tail.
  // |p_new|^2 partials stay per network and are summed in the last segment (norms_and_logs).
  // one GPU: no collective reads a layer's gradient between its weight grad and the optimizer, so the
  // finishes wait for optimize() (MTSAC_DEFER_FINISH=0: each right after its GEMM)
  bool defer_finish() const {
    static const bool on = [] {
      const char* v = getenv("MTSAC_DEFER_FINISH");
      return !(v && atoi(v) == 0);
    }();
    return on && !sharded();
  }

  void optimize(Net& net, float lr, float max_norm, bool polyak, int slot) {
    finish_many(net.fin_sink, net.E, cur);  // the deferred weight-grad finishes (empty when sharded)
    if (zero_of(net)) {
      optimize_zero(net, lr, max_norm, polyak, slot);
      return;
    }
    float* extra = net.g + net.n_flat;
    int gh = 0;
    const int gt = sumsq2(sharded() ? nullptr : net.g, net.trunk_off, net.g + net.trunk_off, net.n_flat - net.trunk_off,
                          net.hparts, net.gparts, net.sc, &gh, cur);
    AdamParams a{}, at{};
    TileParams tp{};
    opt_params(net, lr, polyak, a, at, tp);
    FusedOpt f{};
    f.gparts = net.gparts;
    f.ng = gt;
    f.hparts = net.hparts;
    f.nh = gh;
    f.head_sq = sharded() ? extra + 0 : nullptr;
    f.max_norm = max_norm;
    f.ph = net.pph;
    f.pt = net.ppt;
    adam_fused(a, at, tp, f, cur);
    net.n_pph = f.bh;
    net.n_ppt = f.bt + f.btile;
    wgrid[&net == &critic ? 1 : 0] = f.bh + f.bt + f.btile;
    wbh[&net == &critic ? 1 : 0] = f.bh;
    if (sharded()) sum_partials(net.pph, f.bh, pn + 2 + slot, cur);  // the heads' |p|^2, all-reduced later
  }

  // Sharded trunk optimizer (ZeRO-1 style, mtsac_set_sharded_optimizer).  The trunk buckets were
  // reduce-scattered (backward_segs, reduce_rest); the heads' |g|^2 is in the scalar tail (head_sq).
  //   1. |g|^2 of this rank's shards into the tail, the tail all-reduced: the global clip norm;
  //   2. Adam on the heads (+ their Polyak) and on this rank's trunk shards only (fp32, no planes);
  //   3. the new trunk all-gathered, bucket by bucket;
  //   4. a refresh pass over heads and trunk without the Adam step: the trunk's Polyak target, the GEMM
  //      planes, |p_new|^2 partials and (split2h) weight maxima, exactly as the fused optimizer leaves them.
  void optimize_zero(Net& net, float lr, float max_norm, bool polyak, int slot) {
    float* extra = net.g + net.n_flat;
    const int W = coll_world(), R = coll_rank();
    long long bb[MAXD + 1], be[MAXD + 1];
    const int nb = zero_buckets(net, bb, be);
    ShardRanges sr{};
    long long lo[MAXD + 1], hi[MAXD + 1];  // this rank's shards, relative to the trunk start (floats)
    for (int k = 0; k < nb; ++k) {
      const long long sh = (be[k] - bb[k]) / W;
      lo[k] = bb[k] + R * sh - net.trunk_off;
      hi[k] = lo[k] + sh;
      sr.b[k] = (bb[k] + R * sh) / 4;
      sr.e[k] = (bb[k] + R * sh + sh) / 4;
    }
    sr.n = nb;
    shard_sumsq_add(net.g, sr, zparts, extra + 0, net.sc, cur);  // bumps the Adam count too
    allreduce(extra, (size_t)EXTRA);
    AdamParams a{}, at{};
    TileParams tp{};
    opt_params(net, lr, polyak, a, at, tp);
    // 2. the shard update: heads as always; the trunk elementwise over the shards only (everything else
    // skipped), no tiles, no planes, no Polyak, no maxima
    AdamParams as = at;
    as.target = nullptr;
    as.nseg = 0;
    as.h2 = WeightH2{};
    as.nskip = 0;
    {
      int ord[MAXD + 1];
      for (int k = 0; k < nb; ++k) ord[k] = k;
      std::sort(ord, ord + nb, [&](int x, int y) { return lo[x] < lo[y]; });
      long long prev = 0;
      for (int q = 0; q < nb; ++q) {
        const int k = ord[q];
        if (lo[k] > prev) {
          if (as.nskip >= MAX_PLANE_SEGS) {  // zero_ok admits at most MAX_PLANE_SEGS - 1 buckets
            comm_error = "sharded optimizer: too many skip ranges";
            return;
          }
          as.skip_b[as.nskip] = prev / 4;
          as.skip_e[as.nskip++] = lo[k] / 4;
        }
        prev = hi[k];
      }
      const long long n = net.n_flat - net.trunk_off;
      if (prev < n) {
        if (as.nskip >= MAX_PLANE_SEGS) {
          comm_error = "sharded optimizer: too many skip ranges";
          return;
        }
        as.skip_b[as.nskip] = prev / 4;
        as.skip_e[as.nskip++] = (n + 3) / 4;
      }
    }
    AdamParams ah = a;
    ah.h2 = WeightH2{};
    TileParams none{};
    FusedOpt f{};
    f.head_sq = extra + 0;  // the all-reduced heads + trunk |g|^2
    f.max_norm = max_norm;
    f.ph = zscr;
    f.pt = zscr + FUSED_HEAD_PARTS;
    adam_fused(ah, as, none, f, cur);
    // 3. the new trunk from its owners
    for (int k = nb - 1; k >= 0; --k) coll(2, net.p + bb[k], (size_t)(be[k] - bb[k]));  // layer 0 first
    // 4. refresh: no Adam step; heads without Polyak (done above), the trunk with it
    AdamParams hr = a, tr = at;
    hr.refresh = 1;
    hr.target = nullptr;
    tr.refresh = 1;
    FusedOpt g{};
    g.head_sq = extra + 0;
    g.max_norm = max_norm;
    g.ph = net.pph;
    g.pt = net.ppt;
    adam_fused(hr, tr, tp, g, cur);
    net.n_pph = g.bh;
    net.n_ppt = g.bt + g.btile;
    wgrid[&net == &critic ? 1 : 0] = g.bh + g.bt + g.btile;
    wbh[&net == &critic ? 1 : 0] = g.bh;
    if (sharded()) sum_partials(net.pph, g.bh, pn + 2 + slot, cur);
  }

  // the fused optimizer's operands of one network: heads (a), trunk elementwise leaves (at) and the
  // trunk's kernel tiles with their planes (tp)
  void opt_params(Net& net, float lr, bool polyak, AdamParams& a, AdamParams& at, TileParams& tp) {
    a = AdamParams{};
    a.p = net.p;
    a.m = net.m;
    a.v = net.v;
    a.g = net.g;
    a.target = polyak ? net.tgt : nullptr;
    a.lr = lr;
    a.b1 = cfg.adam_b1;
    a.b2 = cfg.adam_b2;
    a.eps = cfg.adam_eps;
    a.tau = cfg.tau;
    a.sc = net.sc;
    a.np = np;
    if (h2) {
      const int w = &net == &critic ? 1 : 0;
      a.h2.wrec = w_rec(net, 0).d;
      a.h2.trec = polyak ? w_rec(net, 1).d : nullptr;
      a.h2.w_add = adam_step_bound() * lr;
      a.h2.wparts = wparts[w];
      a.h2.tparts = polyak ? tparts : nullptr;
    }
    a.n = net.trunk_off;  // heads
    if (whT_fused(net)) {
      a.whT = net.whT;
      a.whT_b4 = net.off_hW / 4;
      a.whT_e4 = (net.off_hW + (long long)T_l * net.width * net.hd) / 4;
      a.whT_W = net.width;
      a.whT_hd = net.hd;
    }
    at = a;               // trunk
    at.whT = nullptr;
    at.p += net.trunk_off;
    at.m += net.trunk_off;
    at.v += net.trunk_off;
    at.g += net.trunk_off;
    if (at.target) at.target += net.trunk_off;
    at.n = net.n_flat - net.trunk_off;
    tp = TileParams{};
    if (tiles_fusable(net)) {  // kernel leaves in tiles: natural + transposed planes from the update
      for (int i = 0; i < net.depth; ++i) {
        TileLeaf& lf = tp.leaf[tp.n++];
        lf.off = net.off_W[i] - net.trunk_off;
        lf.ms = net.ms_W[i];
        lf.rows = i == 0 ? net.in_dim : net.width;
        lf.cols = net.width;
        lf.members = net.E;
        lf.tiles_r = (lf.rows + 63) / 64;
        lf.tiles_c = (lf.cols + 63) / 64;
        lf.tile_begin = tp.total;
        tp.total += lf.tiles_r * lf.tiles_c * lf.members;
        lf.nat[0] = i > 0 ? net.wp[0][i] : nullptr;  // the data grad's B (layer 0 has none)
        lf.nat_ld = net.wld;
        lf.nat_ps = net.kps(i);
        lf.tr[0] = net.wtp[0][i];
        lf.tr[1] = polyak ? net.wtp[1][i] : nullptr;
        lf.tr_ld = net.wtk(i);
        lf.tr_ps = net.wtps(i);
        lf.frag = net.bfrag[i] ? 1 : 0;
        at.skip_b[at.nskip] = lf.off / 4;
        at.skip_e[at.nskip++] = (lf.off + lf.ms * net.E) / 4;
      }
    } else if (planes_fusable(net)) {  // hidden kernels' planes (params and Polyak target) from the update
      for (int i = 0; i < net.depth && at.nseg + 2 <= MAX_PLANE_SEGS; ++i) {
        at.seg[at.nseg++] = PlaneSeg{net.off_W[i] - net.trunk_off, net.ms_W[i], net.E, net.wp[0][i], net.kps(i), 0};
        if (polyak)
          at.seg[at.nseg++] = PlaneSeg{net.off_W[i] - net.trunk_off, net.ms_W[i], net.E, net.wp[1][i], net.kps(i), 1};
      }
    }
  }

  // gemm_x3f / gemm_x3s nets: every plane the GEMMs read comes out of the tiled update
  // (adam_update_tiles): W_i^T planes of params and target, W_i planes of params (i >= 1)
  bool tiles_fusable(const Net& net) const {
    return planes && net.x3f && net.depth <= MAX_TILE_LEAVES && net.width % 4 == 0;
  }

  // the kernel planes can come straight out of the flat update when their layout is the leaf's
  bool planes_fusable(const Net& net) const {
    return planes && net.wld == net.width && net.wrows == net.width && net.depth <= MAX_PLANE_SEGS / 2;
  }

  void head_sq(Net& net) {  // local |g_head|^2 into the scalar tail
    int np = sumsq_partials(net.g, net.trunk_off, partials, PART, cur);
    sum_partials(partials, np, net.g + net.n_flat + 0, cur);
  }

  // ------------------------------------------------------------ step DAG
  // One step = a DAG of segments; a segment is a short single-stream kernel sequence.
  //  * eager: each segment runs on one of 4 lanes (streams); cross-lane edges are events.
  //  * graph build: each segment is captured ALONE (single-stream capture) into a child graph
  //    and added to the step graph with explicit dependency edges.  No multi-stream capture:
  //    the ROCm 7.0 HIP runtime bundled with torch segfaults in hipStreamEndCapture on nested
  //    stream forks (tools/capture_probe.cpp), while child-graph composition works.
  struct Seg {
    hipStream_t lane;
    hipEvent_t ev;
    hipGraphNode_t node;
  };
  std::vector<Seg> segs;
  hipGraph_t build = nullptr;  // non-null while building the step graph

  template <class F>
  int seg(std::initializer_list<int> deps, int lane, F&& body) {
    Seg s{};
    cur_lane = lane;
    if (build) {
      std::vector<hipGraphNode_t> dn;
      for (int d : deps)  // a repeated dependency (s_afs = s_af unsplit) is an invalid graph edge list
        if (std::find(dn.begin(), dn.end(), segs[d].node) == dn.end()) dn.push_back(segs[d].node);
      hipGraph_t g = nullptr;
      hipError_t r = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
      cur = st;
      body();
      hipError_t r2 = hipStreamEndCapture(st, &g);
      if (r == hipSuccess) r = r2;
      if (r == hipSuccess) r = hipGraphAddChildGraphNode(&s.node, build, dn.data(), dn.size(), g);
      if (g) (void)hipGraphDestroy(g);
      if (r != hipSuccess) comm_error = std::string("step graph build: ") + hipGetErrorString(r);
    } else {
      hipStream_t L = timing_serial ? st
                      : one_stream  ? (pf_issue ? s2 : lane == 4 && dev_collective() ? s4 : st)  // collectives keep their stream
                                    : (lane == 0 ? st : lane == 1 ? s1 : lane == 2 ? s2 : lane == 3 ? s3 : s4);
      for (int d : deps)
        if (segs[d].lane != L) {
          if (segs[d].ev == nullptr && !evpool.empty()) {  // recorded lazily (below): record it now --
            segs[d].ev = evpool[ev_next++ % evpool.size()];  // the main stream's work so far covers d
            (void)hipEventRecord(segs[d].ev, segs[d].lane);
          }
          (void)hipStreamWaitEvent(L, segs[d].ev, 0);
        }
      cur = L;
      body();
      s.lane = L;
      if (L == st && one_stream) {
        // one stream: only the collective stream (lane 4, sharded) and the prefetch stream ever wait
        // on a main-stream segment; its event is recorded when such a wait is issued (an event
        // record per segment left ~1.3 us between consecutive kernels)
        s.ev = nullptr;
      } else if (!evpool.empty()) {  // rotating: an event is re-recorded only pool-size segments later
        // lanes: a wrapped pool could re-record an event another lane has yet to wait on
        if (!one_stream && !ev_rotate && ev_next >= evpool.size()) comm_error = "event pool exhausted";
        s.ev = evpool[ev_next++ % evpool.size()];
        (void)hipEventRecord(s.ev, L);
      } else {
        comm_error = "event pool exhausted";
      }
    }
    segs.push_back(s);
    cur = st;
    return (int)segs.size() - 1;
  }

  // trunk backward as segments: data chain on lane 1, weight grads on lane 3
  // With RCCL, each hidden layer's gradient (b_i, W_i: one contiguous trunk range) is all-reduced
  // on lane 4 as soon as its weight grad is done, overlapping the rest of the backward; the
  // buckets form one chain (every rank issues its collectives in the same order).  Layer 0 and
  // the scalar tail follow in the optimizer segment (reduce_rest).
  // pre_join (may be empty): segments issued after the last weight grad and before the join that
  // waits for the all-reduce buckets (the split actor forward, beside the critic's collective)
  template <class PJ = void (*)()>
  int backward_segs(Net& net, const float* params, const float* X, int ldx, float** acts, __bf16** actp, float** dz,
                    __bf16** dzp, int d_top, int w_prev, int M, PJ pre_join = [] {}) {
    int dprev = d_top, wprev = w_prev, rprev = -1;
    const bool bucket = sharded() && net.depth > 1;
    for (int i = net.depth - 1; i >= 0; --i) {
      wprev = seg({dprev, wprev}, 3, [&, i] { wgrad_layer(net, X, ldx, acts, actp, dz, dzp, i, M); });
      if (bucket && i > 0) {
        const long long b = net.off_b[i], e = (i + 1 < net.depth) ? net.off_b[i + 1] : net.n_flat;
        const int op = zero_of(net) ? 1 : 0;  // the sharded optimizer reduce-scatters
        rprev = rprev < 0 ? seg({wprev}, 4, [&, b, e, op] { coll(op, net.g + b, (size_t)(e - b)); })
                          : seg({wprev, rprev}, 4, [&, b, e, op] { coll(op, net.g + b, (size_t)(e - b)); });
      }
      if (i > 0) dprev = seg({dprev}, 1, [&, i] { dgrad_layer(net, params, acts, actp, dz, dzp, i, M); });
    }
    pre_join();
    if (rprev >= 0) return seg({dprev, wprev, rprev}, 1, [] {});  // join point
    return seg({dprev, wprev}, 1, [] {});
  }

  // the trunk-gradient all-reduce left after backward_segs: everything, or (buckets) layer 0 and
  // the scalar tail
  void reduce_rest(Net& net) {
    if (zero_of(net)) {  // layer 0's bucket (the whole trunk of a one-layer net); the tail in optimize_zero
      const long long e = net.depth > 1 ? net.off_b[1] : net.n_flat;
      coll(1, net.g + net.trunk_off, (size_t)(e - net.trunk_off));
      return;
    }
    if (sharded() && net.depth > 1) {
      allreduce(net.g + net.trunk_off, (size_t)(net.off_b[1] - net.trunk_off));
      allreduce(net.g + net.n_flat, (size_t)EXTRA);
    } else {
      allreduce(net.g + net.trunk_off, (size_t)(net.n_flat - net.trunk_off + EXTRA));
    }
  }

  // ------------------------------------------------------------ one gradient step
  // Segments of _update_inner (mtsac.py:1173-1247):
  //   inputs -> { critic(s,a) fwd | actor(s) fwd + pi | actor(s') + target critic -> y }
  //   -> critic loss -> { data-grad chain | weight grads } -> all-reduce, clip/Adam/Polyak
  //   -> critic(s, a~pi) with the UPDATED critic -> action grad -> actor backward
  //   -> all-reduce, clip/Adam, temperature, logs.
  // Independent GEMM chains fill each other's tail waves.  With timing on, everything runs
  // serialised on the main stream so per-launch events measure solo kernels.
  void use_inset(int k) {
    inset_cur = k;
    xa = inset[k].xa;
    xan = xa + actor.krows * ld_a;
    task = inset[k].task;
    counts = inset[k].counts;
    rows = inset[k].rows;
    // the planes alternate with xa: the input-layer weight grad of step k's actor backward reads
    // them (on k-major planes below 4096 rows) after s_ap, while step k + 1's gather writes the other set
    inp[0].x = xa;
    inp[0].p = inset[k].xap;
  }

  // pipelined: eager issue that overlaps the previous step's tail (see InSet); join: the main
  // stream waits for every lane at the end (the last step of a call, and every non-pipelined one)
  void step(bool device_batch, bool device_noise, bool pipelined = false, bool join = true) {
    const int Bl = B;
    pipelined = pipelined && !build && !timing_serial;
    const bool overlap = pipelined && have_prev;
    // one stream (p2): step k's tail keeps the main stream; the overlapped segments go to s2.
    // lanes: step k's tail is on lanes 1, 3, 4 and the overlapped segments start on lane 0.
    const bool p2 = one_stream;
    if (overlap) use_inset(inset_cur ^ 1);
    counts = device_batch ? s_counts : inset[inset_cur].counts;
    rows = device_batch ? s_rows : inset[inset_cur].rows;
    if (!ev_rotate) ev_next = 0;
    segs.clear();
    actor.fin_sink.n = critic.fin_sink.n = 0;  // (a step cut short never leaves deferred finishes behind)
    zstep[0] = zero_ok(actor);
    zstep[1] = zero_ok(critic);
    const float* twp = cfg.use_task_weights ? tw : nullptr;
    PolicyParams pp{};
    pp.seed = cfg.noise_seed;
    pp.counter = counter;
    pp.A = A;
    pp.ls_min = cfg.log_std_min;
    pp.ls_max = cfg.log_std_max;
    pp.ld_a_out = ld_c;
    pp.ap_ps = critic.arows * critic.xld;
    pp.ap_ld = (int)critic.xld;
    pp.counts = counts;
    pp.rows = rows;
    pp.max_rows = Bl;
    pp.T_l = T_l;
    pp.max_count = device_batch ? n : Bl;  // replay batches hold exactly n rows per task
    CriticHeadParams ch{};
    ch.rew = rew;
    ch.done = done;
    ch.log_alpha = log_alpha;
    ch.task = task;
    ch.task_begin = cfg.task_begin;
    ch.tw = twp;
    ch.gamma = cfg.gamma;
    ch.clip = cfg.clip;
    ch.T_glob = T_g;

    if (overlap) {  // the gather and critic(s, a) reuse buffers step k's actor-loss pass reads
      hipStream_t w = p2 ? s2 : st;
      (void)hipStreamWaitEvent(w, ev_ap[step_par ^ 1], 0);
      // log_alpha (row_alpha) and row_c, which step k's tail reads
      if (cfg.use_task_weights) (void)hipStreamWaitEvent(w, ev_tail[step_par ^ 1], 0);
    }
    pf_issue = overlap && p2;
    const int s_in = seg({}, 0, [&] {
      GatherParams gp = gather_params();
      if (device_batch) {
        replay_indices(rng, jump, buf_size, n, idx, cur);
        replay_gather(gp, cur);
      } else {
        if (h2) user_batch_max(gp, Bl);
        batch_scatter(gp, u_obs, u_act, u_nobs, u_done, u_rew, Bl, cur);
        task_rows(task, Bl, T_l, counts, rows, Bl, cur);  // a user batch: lists from its task ids
      }
      if (cfg.use_task_weights) row_alpha(task, cfg.task_begin, log_alpha, T_g, Bl, 1, row_c, tw, cur);
    });
    // critic forward on (s, a) with the current critic (mtsac.py:555); pipelined on lane 2, which
    // the previous step's tail (lanes 1, 3, 4) does not use, so it runs beside that tail
    const bool ol = overlap || lanes_alt;
    const int s_cf = seg({s_in}, ol ? 2 : 1, [&] { trunk_forward(critic, critic.p, 0, xc, ld_c, hc, hcp, Bl); });
    pf_issue = false;
    if (overlap && !p2) (void)hipStreamWaitEvent(st, ev_tail[step_par ^ 1], 0);  // s_af: the updated actor
    // ONE actor forward over [s | s'] with the pre-update actor: update_critic samples a' ~ pi(.|s')
    // (mtsac.py:525-528) and update_actor a ~ pi(.|s) (:640-642) from the same parameters, so the
    // two row blocks share every trunk GEMM (rows krows.. are s'; the pad rows between are zeros)
    // auto: with a device collective, on shards of <= 2048 rows, where the critic's buckets outlast its
    // backward (MT50 at N >= 4); at N = 2 (3200 rows) the buckets hide in the backward and the halved
    // actor GEMMs only cost (profiles/r4l_shard_model_*.txt: N = 8 -58 us, N = 4 -17 us, N = 2 +167 us
    // per step at 300 GB/s)
    const bool split_af = split_actor_req > 0 || (split_actor_req < 0 && dev_collective() && one_stream && !build &&
                                                  !timing_serial && !lanes_alt && Bl <= 2048);
    auto pi_s = [&](PolicyParams& q) {  // pi(s): the actor-loss half of the policy heads
      q = pp;
      q.head = head(actor, actor.p, ha[actor.depth - 1], Bl, task);
      q.eps = device_noise ? nullptr : eps_c;
      q.stream_id = 2;
      q.a_out = xcp;
      q.a_planes = in_planes(xcp);
      q.ap_rec = h2 ? r_in[inset_cur].d : nullptr;
      q.logpi = logpi;
      q.cache = cache;
    };
    const int s_af = seg({s_in}, ol ? 0 : 2, [&] {
      if (split_af) {  // the s' rows only: a' ~ pi(.|s') for the TD target
        trunk_forward(actor, actor.p, 0, xan, ld_a, han, hap_s2, Bl);
        PolicyParams qn = pp;
        qn.head = head(actor, actor.p, han[actor.depth - 1], Bl, task);
        qn.eps = device_noise ? nullptr : eps_n;
        qn.stream_id = 1;
        qn.a_out = xcn;
        qn.a_planes = in_planes(xcn);
        qn.ap_rec = h2 ? r_in[inset_cur].d : nullptr;
        qn.logpi = logpi_n;
        policy_head(qn, cur);
        return;
      }
      trunk_forward(actor, actor.p, 0, xa, ld_a, ha, hap, Ma);
      PolicyParams q = pp;
      q.head = head(actor, actor.p, ha[actor.depth - 1], Bl, task);
      q.eps = device_noise ? nullptr : eps_c;
      q.stream_id = 2;
      q.a_out = xcp;
      q.a_planes = in_planes(xcp);
      q.ap_rec = h2 ? r_in[inset_cur].d : nullptr;
      q.logpi = logpi;
      q.cache = cache;
      PolicyParams qn = pp;
      qn.head = head(actor, actor.p, han[actor.depth - 1], Bl, task);
      qn.eps = device_noise ? nullptr : eps_n;
      qn.stream_id = 1;
      qn.a_out = xcn;
      qn.a_planes = in_planes(xcn);
      qn.ap_rec = q.ap_rec;
      qn.logpi = logpi_n;
      policy_head_pair(q, qn, cur);
      if (snap_on)
        (void)hipMemcpyAsync(dbg_snap[0], ha[actor.depth - 1], sizeof(float) * Ma * actor.width,
                             hipMemcpyDeviceToDevice, cur);
    });
    // target critic at (s', a'), TD target (mtsac.py:529-553)
    const bool fuse_td = one_stream || timing_serial;  // lanes: s_tg and s_cf run on two lanes
    const int s_tg = seg({s_af}, 0, [&] {
      trunk_forward(critic, critic.tgt, 1, xcn, ld_c, hct, hctp, Bl);
      if (!fuse_td) {  // one stream: the TD target rides in the critic loss launch (s_cl)
        CriticHeadParams c = ch;
        c.head = head(critic, critic.tgt, hct[critic.depth - 1], Bl, task);
        c.mode = CH_TARGET;
        c.logpi = logpi_n;
        c.y_out = y;
        critic_head(c, cur);
      }
    });
    // critic loss (mtsac.py:538-566) and head backward
    const HeadParams chp = head(critic, critic.p, hc[critic.depth - 1], Bl, task);
    bool c_both = false;  // the critic head's weight grad went with its data pass (one launch)
    const int s_cl = seg({s_cf, s_tg}, 1, [&] {
      CriticHeadParams c = ch;
      c.head = chp;
      c.mode = CH_CRITIC;
      c.y = y;
      if (fuse_td) {
        c.fused_target = 1;
        c.thead = head(critic, critic.tgt, hct[critic.depth - 1], Bl, task);
        c.logpi = logpi_n;
        c.y_out = y;
      }
      c.dq = dq;
      c.row_a = row_a;
      c.row_b = row_b;
      c.inv_norm = 1.0f / ((float)critic.E * (float)B_glob);
      if (h2) {
        c.dq_rec = r_dq.d;
        c.dq_parts = &r_dq.n;
      }
      critic_head(c, cur);
      c_both = head_bwd_both(critic, chp, dq, Bl, dzcp, true);
      if (!c_both) head_bwd(critic, chp, dq, Bl, dzc, dzcp, true);
      if (sharded()) {  // the loss sums ride in the all-reduced scalar tail (else: step_finish)
        const float* ins[2] = {row_a, row_b};
        reduce_rows(ins, 2, Bl, critic.g + critic.n_flat + 1, cur);
      }
    });
    const int s_chw = seg({s_cl}, 3, [&] {
      if (!c_both)
        head_backward_weight(chp, dq, Bl, counts, rows, Bl, critic.g + critic.off_hW, critic.g + critic.off_hb, cur);
    });
    int s_afs = s_af;
    const int s_cb = backward_segs(critic, critic.p, xc, ld_c, hc, hcp, dzc, dzcp, s_cl, s_chw, Bl, [&] {
      if (split_af)  // the s rows beside the critic's all-reduce
        s_afs = seg({s_in}, 1, [&] {
          trunk_forward(actor, actor.p, 0, xa, ld_a, ha, hap, Bl);
          PolicyParams q;
          pi_s(q);
          policy_head(q, cur);
        });
    });
    // reduce over shards, clip + Adam + Polyak (mtsac.py:599-613)
    const int s_co = seg({s_cb}, 1, [&] {
      if (sharded()) head_sq(critic);  // the heads' |g|^2 into the all-reduced scalar tail
      reduce_rest(critic);
      optimize(critic, cfg.critic_lr, cfg.critic_max_grad_norm, true, 0);
      refresh_wt(critic, critic.p, 0, cur, true);
      refresh_wt(critic, critic.tgt, 1, cur, true);
    });
    // actor loss through the UPDATED critic (mtsac.py:659-691)
    const int s_ap = seg({s_co, s_af, s_afs}, 1, [&] {
      trunk_forward(critic, critic.p, 0, xcp, ld_c, hc, hcp, Bl);
      CriticHeadParams c = ch;
      c.head = head(critic, critic.p, hc[critic.depth - 1], Bl, task);
      c.mode = CH_ACTOR;
      c.logpi = logpi;
      c.dq = dq;
      c.row_a = row_c;
      c.alpha_w = alpha_w;
      c.inv_norm = 1.0f / (float)B_glob;
      if (h2) {
        c.dq_rec = r_dq.d;
        c.dq_parts = &r_dq.n;
      }
      critic_head(c, cur);
      head_bwd(critic, c.head, dq, Bl, dzc, dzcp, false);
      for (int i = critic.depth - 1; i > 0; --i) dgrad_layer(critic, critic.p, hc, hcp, dzc, dzcp, i, Bl, false);
      ActionGradParams ag{};
      ag.dz1 = dzc[0];
      ag.W0 = critic.p + critic.off_W[0];
      ag.s_dz = (long long)Bl * critic.width;
      ag.s_W0 = critic.ms_W[0];
      ag.E = critic.E;
      ag.B = Bl;
      ag.Wc = critic.width;
      ag.A = A;
      ag.cache = cache;
      ag.alpha_w = alpha_w;
      ag.ls_min = cfg.log_std_min;
      ag.ls_max = cfg.log_std_max;
      ag.dout = dout_a;
      if (h2) {
        ag.dout_rec = r_dout.d;
        ag.dout_parts = &r_dout.n;
      }
      action_grad(ag, cur);
      if (snap_on)
        (void)hipMemcpyAsync(dbg_snap[1], ha[actor.depth - 1], sizeof(float) * Ma * actor.width,
                             hipMemcpyDeviceToDevice, cur);
      if (sharded()) {
        const float* ins[1] = {row_c};
        reduce_rows(ins, 1, Bl, actor.g + actor.n_flat + 1, cur);
      }
    });
    if (pipelined) (void)hipEventRecord(ev_ap[step_par], segs[s_ap].lane);
    const HeadParams ahp = head(actor, actor.p, ha[actor.depth - 1], Bl, task);
    // the head's data and weight passes in one launch (head_bwd_both's conditions)
    const bool a_both = top_planes(actor, dzap).p != nullptr && actor.width % 4 == 0;
    const int s_ahw = seg({s_ap}, 3, [&] {
      if (!a_both)
        head_backward_weight(ahp, dout_a, 0, counts, rows, Bl, actor.g + actor.off_hW, actor.g + actor.off_hb, cur);
    });
    const int s_ad = seg({s_ap}, 1, [&] {
      if (!(a_both && head_bwd_both(actor, ahp, dout_a, 0, dzap, true))) head_bwd(actor, ahp, dout_a, 0, dza, dzap, true);
    });
    const int s_ab = backward_segs(actor, actor.p, xa, ld_a, ha, hap, dza, dzap, s_ad, s_ahw, Bl);
    const int s_tail = seg({s_ab}, 1, [&] {
      // temperature gradient rides in the actor's scalar tail: [2] loss part, [3..] grad
      AlphaParams al = alpha_params();
      if (sharded()) alpha_grad(al, cur);  // unsharded: inside step_finish
      if (sharded()) head_sq(actor);
      reduce_rest(actor);
      optimize(actor, cfg.actor_lr, cfg.actor_max_grad_norm, false, 1);
      refresh_wt(actor, actor.p, 0, cur, true);
      // temperature (mtsac.py:713-731), post-update parameter norms (trunk |p|^2 replicated, head
      // |p|^2 summed over shards), logs: one launch
      allreduce(pn + 2, 2);
      StepFinish f{};
      if (!sharded()) {
        f.rows[0] = row_a;
        f.row_out[0] = critic.g + critic.n_flat + 1;
        f.rows[1] = row_b;
        f.row_out[1] = critic.g + critic.n_flat + 2;
        f.rows[2] = row_c;
        f.row_out[2] = actor.g + actor.n_flat + 1;
      }
      f.B = Bl;
      f.alpha = al;
      f.alpha_grad = sharded() ? 0 : 1;
      f.lr = cfg.alpha_lr;
      f.b1 = cfg.adam_b1;
      f.b2 = cfg.adam_b2;
      f.eps = cfg.adam_eps;
      f.max_norm = cfg.alpha_max_grad_norm;
      Net* nets[2] = {&critic, &actor};
      for (int w = 0; w < 2; ++w) {
        f.pn.pt[w] = nets[w]->ppt;
        f.pn.nt[w] = nets[w]->n_ppt;
        f.pn.ph[w] = nets[w]->pph;
        f.pn.nh[w] = nets[w]->n_pph;
        f.pn.sc[w] = nets[w]->sc;
      }
      f.head_sq = sharded() ? pn + 2 : nullptr;
      LogParams& lp = f.logs;
      lp.critic_sums = critic.g + critic.n_flat + 1;
      lp.actor_sums = actor.g + actor.n_flat + 1;
      lp.critic = critic.sc;
      lp.actor = actor.sc;
      lp.alpha_loss_sum = actor.g + actor.n_flat + 2;
      lp.log_alpha = log_alpha;
      lp.T_glob = T_g;
      lp.inv_critic = 1.0f / ((float)critic.E * (float)B_glob);
      lp.inv_actor = 1.0f / (float)B_glob;
      lp.inv_b = 1.0f / (float)B_glob;
      lp.logs = logs;
      f.counter = counter;
      if (h2) {  // the optimizers' weight maxima into the records (the next updates' plane exponents)
        f.wmax[0] = WeightMaxJob{wparts[0], wgrid[0], wbh[0], r_w[0][0].d};
        f.wmax[1] = WeightMaxJob{wparts[1], wgrid[1], wbh[1], r_w[1][0].d};
        f.wmax[2] = WeightMaxJob{tparts, wgrid[1], -1, r_w[1][1].d};
        f.nwmax = 3;
      }
      step_finish(f, cur);
    });
    if (pipelined) (void)hipEventRecord(ev_tail[step_par], segs[s_tail].lane);
    if (!build && (join || !pipelined)) {  // eager: the main stream waits for every lane
      for (const Seg& s : segs)
        if (s.lane != st && s.ev) (void)hipStreamWaitEvent(st, s.ev, 0);
    }
    have_prev = pipelined && !join;
    step_par ^= 1;
    cur = st;
  }

  // ------------------------------------------------------------ per-task gradients (eval metrics)
  // MTSAC.compute_weights (mtsac.py:870-1090, MSE critic): for every task t the gradient of its
  // own loss -- the critic MSE over the task's n rows (mean over E x n), the actor loss over its
  // rows (mean over n) -- w.r.t. the whole network, as dense [T][P] matrices in flax ravel order
  // (leaves back to back, no alignment padding), on the CURRENT parameters (nothing is updated).
  // Kept from the reference: the critic's "next" actions are sampled from pi(.|s) of the
  // OBSERVATIONS (mtsac.py:1000-1004) and scored by the target critic at s' (:1005-1007).
  // Every GEMM here runs on fp32 operands (gemm_x3 / gemm_f32): the per-task weight gradient of
  // layer i is ONE batched TN GEMM over the tasks, X_t^T dZ_t with task t's rows t, t + T, ...
  // addressed by a row stride of T rows (rows interleaved i*T + t, as the buffer samples), its
  // column sums (bias gradient) fused.
  float* tg[2] = {};       // [T][P] critic (0), actor (1)
  long long tgP[2] = {};
  unsigned* sel_prefix = nullptr;
  long long* sel_rank = nullptr;
  unsigned* sel_hist = nullptr;
  double *ps_gram_part = nullptr, *ps_l1_part = nullptr, *ps_gram = nullptr, *ps_l1 = nullptr;
  unsigned long long *ps_counts = nullptr, *ps_nz = nullptr;
  float* ps_thr = nullptr;
  static constexpr int PS_GRID = 512;

  static std::vector<long long> dense_offsets(const Net& net) {  // flax leaf offsets, no padding
    std::vector<long long> off;
    long long o = 0;
    for (const auto& lf : net.leaves) {
      off.push_back(o);
      o += lf.second;
    }
    off.push_back(o);
    return off;
  }

  int ensure_task_grad_buffers() {
    int rc = 0;
    for (int w = 0; w < 2; ++w) {
      const Net& net = w == 0 ? critic : actor;
      tgP[w] = net.n_params;
      if (!tg[w] && (rc = alloc(&tg[w], (size_t)T_l * tgP[w]))) return rc;
    }
    if (!sel_prefix) {
      if ((rc = alloc(&sel_prefix, 2 * 64)) || (rc = alloc(&sel_rank, 2 * 64)) || (rc = alloc(&sel_hist, 512 * 64)) ||
          (rc = alloc(&ps_gram_part, (size_t)PS_GRID * 64 * 64)) || (rc = alloc(&ps_l1_part, (size_t)PS_GRID * 64)) ||
          (rc = alloc(&ps_gram, 64 * 64)) || (rc = alloc(&ps_l1, 64)) || (rc = alloc(&ps_counts, 4 * 64 * 64)) ||
          (rc = alloc(&ps_nz, 64)) || (rc = alloc(&ps_thr, 64)))
        return rc;
    }
    // alloc()'s null-stream zero fills before the engine streams use the buffers
    return hipDeviceSynchronize() == hipSuccess ? 0 : fail(-5, "device synchronize");
  }

  // dW_t, db_t of trunk layer i for every task t (one batched TN GEMM per ensemble member)
  void task_wgrad(Net& net, int w, const float* X, int ldx, float** acts, float** dz, int i) {
    const std::vector<long long> off = dense_offsets(net);
    const int fan = i == 0 ? net.in_dim : net.width;
    const int n_rows = B / T_l;
    for (int e = 0; e < net.E; ++e) {
      GemmParams g{};
      g.A = i == 0 ? X : acts[i - 1] + (long long)e * B * net.width;
      g.lda = (i == 0 ? ldx : net.width) * T_l;
      g.sA = i == 0 ? ldx : net.width;
      g.B = dz[i] + (long long)e * B * net.width;
      g.ldb = net.width * T_l;
      g.sB = net.width;
      g.C = tg[w] + off[3 + 2 * i] + (long long)e * fan * net.width;
      g.ldc = net.width;
      g.sC = tgP[w];
      g.db = tg[w] + off[2 + 2 * i] + (long long)e * net.width;
      g.sDb = tgP[w];
      g.M = fan;
      g.N = net.width;
      g.K = n_rows;
      g.splits = 1;
      gemm(g, GEMM_TN, EPI_STORE, T_l, MTSAC_FAM_WEIGHT_GRAD);
    }
  }

  // the task's own head block (bias, kernel) of the padded gradient buffer into its dense row
  void task_heads(Net& net, int w) {
    const std::vector<long long> off = dense_offsets(net);
    scatter_task_blocks(net.g, net.off_hb, net.ms_hb, tg[w], tgP[w], off[0], (long long)T_l * net.hd, net.E, T_l,
                        net.hd, cur);
    scatter_task_blocks(net.g, net.off_hW, net.ms_hW, tg[w], tgP[w], off[1], (long long)T_l * net.width * net.hd,
                        net.E, T_l, (long long)net.width * net.hd, cur);
  }

  void task_grads(bool device_batch, bool device_noise) {
    const int Bl = B, n_rows = B / T_l;
    cur = st;
    cur_lane = 0;
    counts = inset[inset_cur].counts;  // task_rows below (check_interleaved holds the layout)
    rows = inset[inset_cur].rows;
    GatherParams gp = gather_params();
    if (device_batch) {
      replay_indices(rng, jump, buf_size, n, idx, cur);
      replay_gather(gp, cur);
    } else {
      if (h2) user_batch_max(gp, Bl);
      batch_scatter(gp, u_obs, u_act, u_nobs, u_done, u_rew, Bl, cur);
    }
    check_interleaved(task, Bl, T_l, err, cur);
    task_rows(task, Bl, T_l, counts, rows, Bl, cur);
    if (cfg.use_task_weights) row_alpha(task, cfg.task_begin, log_alpha, T_g, Bl, 1, row_c, tw, cur);
    const float* twp = cfg.use_task_weights ? tw : nullptr;
    for (int w = 0; w < 2; ++w) (void)hipMemsetAsync(tg[w], 0, sizeof(float) * T_l * tgP[w], cur);
    PolicyParams pp{};
    pp.seed = cfg.noise_seed;
    pp.counter = counter;
    pp.A = A;
    pp.ls_min = cfg.log_std_min;
    pp.ls_max = cfg.log_std_max;
    pp.ld_a_out = ld_c;
    pp.counts = counts;
    pp.rows = rows;
    pp.max_rows = Bl;
    pp.T_l = T_l;
    pp.max_count = n_rows;
    CriticHeadParams ch{};
    ch.rew = rew;
    ch.done = done;
    ch.log_alpha = log_alpha;
    ch.task = task;
    ch.task_begin = cfg.task_begin;
    ch.tw = twp;
    ch.gamma = cfg.gamma;
    ch.clip = cfg.clip;
    ch.T_glob = T_g;
    const int Dc = critic.depth, Da = actor.depth;

    // ---- critic (mtsac.py:1000-1048): a_n ~ pi(.|s), y from the target critic at (s', a_n)
    trunk_forward(actor, actor.p, 0, xa, ld_a, han, nullptr, Bl);
    {
      PolicyParams q = pp;
      q.head = head(actor, actor.p, han[Da - 1], Bl, task);
      q.eps = device_noise ? nullptr : eps_n;
      q.stream_id = 3;
      q.a_out = xcn;
      q.logpi = logpi_n;
      policy_head(q, cur);
    }
    trunk_forward(critic, critic.tgt, 1, xcn, ld_c, hct, nullptr, Bl);
    {
      CriticHeadParams c = ch;
      c.head = head(critic, critic.tgt, hct[Dc - 1], Bl, task);
      c.mode = CH_TARGET;
      c.logpi = logpi_n;
      c.y_out = y;
      critic_head(c, cur);
    }
    trunk_forward(critic, critic.p, 0, xc, ld_c, hc, nullptr, Bl);
    const HeadParams chp = head(critic, critic.p, hc[Dc - 1], Bl, task);
    {
      CriticHeadParams c = ch;
      c.head = chp;
      c.mode = CH_CRITIC;
      c.y = y;
      c.dq = dq;
      c.row_a = row_a;
      c.row_b = row_b;
      c.inv_norm = 1.0f / ((float)critic.E * (float)n_rows);  // per-task mean over E x n
      critic_head(c, cur);
    }
    head_backward_data(chp, dq, Bl, dzc[Dc - 1], counts, rows, Bl, T_l, cur);
    head_backward_weight(chp, dq, Bl, counts, rows, Bl, critic.g + critic.off_hW, critic.g + critic.off_hb, cur);
    task_heads(critic, 0);
    for (int i = Dc - 1; i >= 0; --i) {
      task_wgrad(critic, 0, xc, ld_c, hc, dzc, i);
      if (i > 0) dgrad_layer(critic, critic.p, hc, nullptr, dzc, nullptr, i, Bl);
    }

    // ---- actor (mtsac.py:1051-1090): the current critic, per-task mean over n rows
    trunk_forward(actor, actor.p, 0, xa, ld_a, ha, nullptr, Bl);
    {
      PolicyParams q = pp;
      q.head = head(actor, actor.p, ha[Da - 1], Bl, task);
      q.eps = device_noise ? nullptr : eps_c;
      q.stream_id = 4;
      q.a_out = xcp;
      q.logpi = logpi;
      q.cache = cache;
      policy_head(q, cur);
    }
    trunk_forward(critic, critic.p, 0, xcp, ld_c, hc, nullptr, Bl);
    {
      CriticHeadParams c = ch;
      c.head = head(critic, critic.p, hc[Dc - 1], Bl, task);
      c.mode = CH_ACTOR;
      c.logpi = logpi;
      c.dq = dq;
      c.row_a = row_c;
      c.alpha_w = alpha_w;
      c.inv_norm = 1.0f / (float)n_rows;
      critic_head(c, cur);
      head_backward_data(c.head, dq, Bl, dzc[Dc - 1], counts, rows, Bl, T_l, cur);
    }
    for (int i = Dc - 1; i > 0; --i) dgrad_layer(critic, critic.p, hc, nullptr, dzc, nullptr, i, Bl);
    {
      ActionGradParams ag{};
      ag.dz1 = dzc[0];
      ag.W0 = critic.p + critic.off_W[0];
      ag.s_dz = (long long)Bl * critic.width;
      ag.s_W0 = critic.ms_W[0];
      ag.E = critic.E;
      ag.B = Bl;
      ag.Wc = critic.width;
      ag.A = A;
      ag.cache = cache;
      ag.alpha_w = alpha_w;
      ag.ls_min = cfg.log_std_min;
      ag.ls_max = cfg.log_std_max;
      ag.dout = dout_a;
      action_grad(ag, cur);
    }
    const HeadParams ahp = head(actor, actor.p, ha[Da - 1], Bl, task);
    head_backward_data(ahp, dout_a, 0, dza[Da - 1], counts, rows, Bl, T_l, cur);
    head_backward_weight(ahp, dout_a, 0, counts, rows, Bl, actor.g + actor.off_hW, actor.g + actor.off_hb, cur);
    task_heads(actor, 1);
    for (int i = Da - 1; i >= 0; --i) {
      task_wgrad(actor, 1, xa, ld_a, ha, dza, i);
      if (i > 0) dgrad_layer(actor, actor.p, ha, nullptr, dza, nullptr, i, Bl);
    }
  }

  AlphaParams alpha_params() {
    AlphaParams al{};
    al.logpi = logpi;
    al.counts = counts;
    al.rows = rows;
    al.max_rows = B;
    al.T_l = T_l;
    al.task_begin = cfg.task_begin;
    al.T_glob = T_g;
    al.B_glob = B_glob;
    al.target_entropy = -(float)A;
    al.log_alpha = log_alpha;
    al.m = la_m;
    al.v = la_v;
    al.grad = actor.g + actor.n_flat + 3;
    al.loss_part = actor.g + actor.n_flat + 2;
    al.task_loss = alpha_tmp;
    al.sc = sc_alpha;
    return al;
  }

  // split2h, a user batch: its own max |value| bounds the input planes (the stored rows' does not)
  void user_batch_max(GatherParams& gp, int Bl) {
    (void)hipMemsetAsync(ubmax, 0, sizeof(float), cur);
    absmax_into(u_obs, (long long)Bl * D, ubmax, cur);
    absmax_into(u_nobs, (long long)Bl * D, ubmax, cur);
    absmax_into(u_act, (long long)Bl * A, ubmax, cur);
    gp.in_max = ubmax;
  }

  GatherParams gather_params() {
    GatherParams gp{};
    gp.store = store;
    gp.idx = idx;
    gp.n = n;
    gp.T_l = T_l;
    gp.R = R;
    gp.obs_dim = D;
    gp.act_dim = A;
    gp.T_glob = T_g;
    gp.task_begin = cfg.task_begin;
    gp.ld_a = ld_a;
    gp.ld_c = ld_c;
    gp.xa = xa;
    gp.xa_next = xan;
    gp.xc = xc;
    gp.xc_next = xcn;
    gp.xc_pi = xcp;
    gp.rew = rew;
    gp.done = done;
    gp.task = task;
    gp.rmin = cfg.normalize_rewards ? rmin : nullptr;
    gp.rmax = cfg.normalize_rewards ? rmax : nullptr;
    // mode 2 (return normalisation, buffers.py:392-422): rmin = 0, rmax = the per-task denominator
    // set by the host, so (r - 0) / (den - 0 + 0) = r / den in float64
    gp.norm_eps = cfg.normalize_rewards == 2 ? 0.0 : 1e-8;
    gp.err = err;
    if (h2) {
      gp.in_rec = r_in[inset_cur].d;
      gp.in_max = bufmax;
    }
    if (planes) {
      gp.pa = inp[0].p;
      gp.pa_ps = actor.arows * actor.xld;
      gp.pa_ld = (int)actor.xld;
      gp.pa_next = actor.krows;
      gp.pc = in_planes(xc);
      gp.pcn = in_planes(xcn);
      gp.pcp = in_planes(xcp);
      gp.pc_ps = critic.arows * critic.xld;
      gp.pc_ld = (int)critic.xld;
    }
    return gp;
  }

  int check_err() {
    if (!comm_error.empty()) {
      std::string m = comm_error;
      comm_error.clear();
      return fail(-5, m);
    }
    int e[2] = {0, 0};  // [0] the batch check, [1] the head backward's self-check bits (HEAD_FAULT_*)
    HIP_TRY(hipMemcpyAsync(e, err, sizeof(e), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (e[0] || e[1]) {
      const int z[2] = {0, 0};
      HIP_TRY(hipMemcpy(err, z, sizeof(z), hipMemcpyHostToDevice));
    }
    if (e[1])
      return fail(-5, std::string("head backward self-check failed (bits ") + std::to_string(e[1]) +
                          "): a cross-wave LDS reduction slot held other bits than its writer stored, so this "
                          "step's head gradients are not trustworthy (DESIGN.md section 5)");
    if (e[0])
      return fail(-22,
                  "batch rows must end in an exact one-hot task id owned by this engine (obs and next_obs agree)");
    return 0;
  }
};

// ================================================================ C-ABI
extern "C" {

const char* mtsac_last_error(void) { return g_last_error.c_str(); }
int mtsac_abi_version(void) { return MTSAC_ABI_VERSION; }

void mtsac_default_config(mtsac_config* c, int32_t T) {
  std::memset(c, 0, sizeof(*c));
  c->num_tasks = T;
  c->task_begin = 0;
  c->task_count = T;
  c->obs_dim = 39 + T;
  c->action_dim = 4;
  c->actor_width = 400;
  c->actor_depth = 3;
  c->critic_width = 400;
  c->critic_depth = 3;
  c->num_critics = 2;
  c->batch_per_task = 128;
  c->capacity = 100000;
  c->gamma = 0.99f;
  c->tau = 0.005f;
  c->actor_lr = c->critic_lr = c->alpha_lr = 3e-4f;
  c->actor_max_grad_norm = 1.0f;
  c->critic_max_grad_norm = 1.0f;
  c->alpha_max_grad_norm = -1.0f;  // None: no clip (mtsac.py:120)
  c->adam_b1 = 0.9f;
  c->adam_b2 = 0.999f;
  c->adam_eps = 1e-5f;
  c->initial_temperature = 1.0f;
  c->log_std_min = -20.0f;
  c->log_std_max = 2.0f;
  c->precision = MTSAC_FP32;
  c->noise_seed = 2;
}

int pcg_jump_table(unsigned long long* out /* 65*4 */) {
  // state_{j} = A_j s + C_j inc;  A_0 = 1, C_0 = 0;  A_{j+1} = M A_j, C_{j+1} = M C_j + 1
  typedef unsigned __int128 u128h;
  const u128h M = ((u128h)0x2360ED051FC65DA4ull << 64) | (u128h)0x4385DF649FCCF645ull;
  u128h a = 1, c = 0;
  for (int j = 0; j <= 64; ++j) {
    out[4 * j + 0] = (unsigned long long)(a >> 64);
    out[4 * j + 1] = (unsigned long long)a;
    out[4 * j + 2] = (unsigned long long)(c >> 64);
    out[4 * j + 3] = (unsigned long long)c;
    a = a * M;
    c = c * M + 1;
  }
  return 0;
}

int mtsac_create(const mtsac_config* cfg, int hip_device, mtsac_engine** out) {
  if (!cfg || !out) return fail(-22, "null argument");
  *out = nullptr;
  const mtsac_config& c = *cfg;
  if (c.num_tasks < 1 || c.task_count < 1 || c.task_begin < 0 || c.task_begin + c.task_count > c.num_tasks)
    return fail(-22, "invalid task range");
  if (c.task_count > 64) return fail(-22, "at most 64 tasks per engine");
  if (c.num_tasks > EXTRA - 8) return fail(-22, "num_tasks too large");
  if (c.action_dim < 1 || c.action_dim > 4) return fail(-22, "action_dim must be in [1, 4]");
  if (c.obs_dim < c.num_tasks) return fail(-22, "obs_dim must include the one-hot task id");
  if (c.actor_width % 4 || c.critic_width % 4 || c.actor_width <= 0 || c.critic_width <= 0)
    return fail(-22, "network widths must be positive multiples of 4");
  if (c.actor_depth < 1 || c.actor_depth > MAXD || c.critic_depth < 1 || c.critic_depth > MAXD)
    return fail(-22, "depth must be in [1, 8]");
  if (c.num_critics < 1 || c.num_critics > 4) return fail(-22, "num_critics must be in [1, 4]");
  if (c.batch_per_task < 1) return fail(-22, "batch_per_task must be positive");
  if (c.normalize_rewards < 0 || c.normalize_rewards > 2) return fail(-22, "normalize_rewards must be 0, 1 or 2");
  if (c.capacity < c.batch_per_task || c.capacity >= (1ll << 31))
    return fail(-22, "capacity must be in [batch_per_task, 2^31)");
  if (c.precision != MTSAC_FP32 && c.precision != MTSAC_FP32_SPLIT3 && c.precision != MTSAC_BF16 &&
      c.precision != MTSAC_FP32_SPLIT2H)
    return fail(-22, "unsupported precision");
  if (c.precision == MTSAC_FP32_SPLIT2H && (long long)c.batch_per_task * c.task_count > 8192)
    return fail(-22, "split2h: at most 8192 rows per engine (the sizes its partial-maximum records and plane bounds are validated at; precision split3 has no such limit)");
  if (c.precision == MTSAC_FP32_SPLIT2H && !(c.adam_b1 * c.adam_b1 < c.adam_b2))
    return fail(-22, "split2h bounds an Adam step (|m_hat| / sqrt(v_hat)), which needs adam_b1^2 < adam_b2");
  hipError_t he = hipSetDevice(hip_device);
  if (he != hipSuccess) return fail(-19, std::string("hipSetDevice: ") + hipGetErrorString(he));

  auto* e = new mtsac_engine();
  e->geo_at_create = g_x3p_geo;
  e->cfg = c;
  e->device = hip_device;
  e->T_l = c.task_count;
  e->T_g = c.num_tasks;
  e->A = c.action_dim;
  e->D = c.obs_dim;
  e->n = c.batch_per_task;
  e->B = c.batch_per_task * c.task_count;
  {
    const char* v = getenv("MTSAC_INPUT_WGRAD");
    // split2h planes are 4 B per element, as the fp32 dz[0] is: planes everywhere (S3 -54 us per step,
    // profiles/r5n_step_ab.txt); split3's 6 B per element pay only below 4096 rows
    e->in_wgrad_planes = v ? atoi(v) != 0 : (e->B < 4096 || c.precision == MTSAC_FP32_SPLIT2H);
  }
  e->B_glob = c.batch_per_task * c.num_tasks;
  e->R = (int)align_up(2LL * e->D + e->A + 2, 4);
  e->ld_a = (int)align_up(e->D, 4);
  e->ld_c = (int)align_up(e->D + e->A, 4);
  e->roll_max = std::max(64, c.num_tasks);
  int rc = 0;
  auto bad = [&](int r) {
    delete e;
    return r;
  };
  // Streams: the main stream, the prefetch stream s2, the collective stream s4 and the buffer-add pack
  // stream sa -- four, so HIP's default four hardware queues give each its own.  s1 and s3 serve only
  // the experimental 5-lane form and exist only when it is requested (MTSAC_LANES=1).  Streams beyond
  // GPU_MAX_HW_QUEUES share hardware queues, and concurrently active streams on a shared queue were
  // seen to read stale data ("Lanes and hardware queues").
  {
    const char* lw = getenv("MTSAC_LANES");
    const bool lanes_wanted = lw && atoi(lw) != 0;
    // diagnostics (MTSAC_CU_SLICE=k:n): this engine's streams run on CU slice k of n only, so engines
    // sharing one device in a test never share a CU
    std::vector<uint32_t> cu_mask;
    if (const char* cs = getenv("MTSAC_CU_SLICE")) {
      int k = 0, n = 1, ncu = 0;
      if (sscanf(cs, "%d:%d", &k, &n) == 2 && n >= 1 && k >= 0 && k < n &&
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, hip_device) == hipSuccess && ncu > 0) {
        cu_mask.assign((ncu + 31) / 32, 0u);
        for (int c = k * ncu / n; c < (k + 1) * ncu / n; ++c) cu_mask[c / 32] |= 1u << (c % 32);
      }
    }
    for (hipStream_t* x : {&e->st, &e->s2, &e->s4, &e->sa, &e->s1, &e->s3}) {
      if ((x == &e->s1 || x == &e->s3) && !lanes_wanted) continue;
      const hipError_t r = cu_mask.empty()
                               ? hipStreamCreateWithFlags(x, hipStreamNonBlocking)
                               : hipExtStreamCreateWithCUMask(x, (uint32_t)cu_mask.size(), cu_mask.data());
      if (r != hipSuccess) return bad(fail(-5, "stream"));
    }
  }
  e->lane_mode_for();
  e->cur = e->st;
  for (int i = 0; i < 128; ++i) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return bad(fail(-5, "event"));
    e->evpool.push_back(ev);
  }

  e->actor.layout(e->D, e->ld_a, c.actor_width, c.actor_depth, e->T_l, 2 * e->A, 1);
  e->critic.layout(e->D + e->A, e->ld_c, c.critic_width, c.critic_depth, e->T_l, 1, c.num_critics);
  for (Net* net : {&e->actor, &e->critic}) {
    if ((rc = e->alloc(&net->p, net->n_flat))) return bad(rc);
    if ((rc = e->alloc(&net->g, net->n_flat + EXTRA))) return bad(rc);
    if ((rc = e->alloc(&net->m, net->n_flat))) return bad(rc);
    if ((rc = e->alloc(&net->v, net->n_flat))) return bad(rc);
    if ((rc = e->alloc(&net->sc, 1))) return bad(rc);
    if ((rc = e->alloc(&net->gparts, 1024)) || (rc = e->alloc(&net->hparts, FUSED_HEAD_PARTS)) ||
        (rc = e->alloc(&net->pph, FUSED_HEAD_PARTS)) || (rc = e->alloc(&net->ppt, 2048)))
      return bad(rc);
  }
  if ((rc = e->alloc(&e->critic.tgt, e->critic.n_flat))) return bad(rc);
  e->planes = c.precision == MTSAC_FP32_SPLIT3 || c.precision == MTSAC_BF16 || c.precision == MTSAC_FP32_SPLIT2H;
  e->np = c.precision == MTSAC_BF16 ? 1 : c.precision == MTSAC_FP32_SPLIT2H ? 2 : 3;
  e->h2 = c.precision == MTSAC_FP32_SPLIT2H;
  if (e->h2) e->adam_bound = mtsac_engine::adam_step_bound_of(c.adam_b1, c.adam_b2);
  if (e->h2) {  // the plane records, the stored rows' bound, the optimizer's maxima
    const int nrec = 2 + 4 + 3 * MAXD + 2 * MAXD + 2;
    if ((rc = e->alloc(&e->recs, (size_t)nrec))) return bad(rc);
    PlaneRec* r = e->recs;
    for (auto& x : e->r_in) x.d = r++;
    for (auto& w : e->r_w)
      for (auto& x : w) x.d = r++;
    for (auto& a : e->r_ac)
      for (auto& x : a) x.d = r++;
    for (auto& a : e->r_dz)
      for (auto& x : a) x.d = r++;
    e->r_dq.d = r++;
    e->r_dout.d = r++;
    if ((rc = e->alloc(&e->bufmax, 1)) || (rc = e->alloc(&e->ubmax, 1)) || (rc = e->alloc(&e->wparts[0], 4096)) ||
        (rc = e->alloc(&e->wparts[1], 4096)) || (rc = e->alloc(&e->tparts, 4096)))
      return bad(rc);
  }
  for (Net* net : {&e->actor, &e->critic}) {
    net->wld = align_up(net->width, 32);
    net->wrows = align_up(net->width, 32);
    net->ald = align_up(net->width, 32);
    net->xld = align_up(net->in_dim, 32);
    net->krows = align_up(e->B, 32);
    net->arows = net == &e->actor ? align_up(net->krows + e->B, 32) : net->krows;
    // row-major x row-major plane GEMMs for the trunk forward and data grad (hidden activations
    // then keep planes only): gemm_x3f when its 208 x 256 tiles fill the chip (with split-K when
    // they do not), gemm_x3s for narrow trunks (K <= 512: W = 400).  The 16 TI x 64 tiles of
    // gemm_x3s are bound by the per-CU operand ingest on wide trunks (texture-address unit busy
    // 94 %, tools/x3s_ablate.py), and narrow trunks on many rows (MT50 at
    // W = 400) run faster on gemm_x3p's 256 x 128 tiles.
    // Task shards of wide trunks (B = 768..1280 at W = 2048): gemm_x3f + split-K beats gemm_x3p +
    // split-K for the twin critic (E = 2: 64-80 row x column tiles, 8-20 % per launch,
    // tools/x3f_split_bench.py) but not for the actor (E = 1), which stays on gemm_x3p.
    static const int x3f_min_tiles = [] {  // MTSAC_X3F_MIN_TILES: experiments
      const char* v = getenv("MTSAC_X3F_MIN_TILES");
      return v ? atoi(v) : 64;
    }();
    const int M_fwd = net == &e->actor ? (int)(net->krows + e->B) : e->B;  // the actor forward's rows
    net->x3f = e->planes && net->depth > 1 &&
               ((net->ald % 64 == 0 && gemm_x3f_tiles(M_fwd, net->width, net->E) >= x3f_min_tiles) ||
                (net->ald <= 512 && e->B <= 2048));
    if (net->x3f) net->xld = align_up(net->in_dim, 64);  // gemm_x3f steps K by 64
    static const int bfrag_env = [] {  // MTSAC_BFRAG=0: row-major weight planes (experiments)
      const char* v = getenv("MTSAC_BFRAG");
      return v ? atoi(v) : 1;
    }();
    const int bfrag_req = g_bfrag_mode >= 0 ? g_bfrag_mode : bfrag_env;
    // candidates; frag_probe (after the workspaces) keeps those whose every trunk GEMM is gemm_x3f's
    const bool cand = net->x3f && bfrag_req != 0 && net->depth <= MAX_TILE_LEAVES && net->width % 16 == 0 &&
                      net->ald % 64 == 0 && net->wld % 32 == 0;
    for (int i = 0; i < net->depth; ++i) net->bfrag[i] = cand;
    for (int w = 0; w < (net == &e->critic ? 2 : 1); ++w)
      for (int i = 0; i < net->depth; ++i) {
        if (!e->planes) {
          if (i > 0 && (rc = e->alloc(&net->wt[w][i], (size_t)net->ms_W[i] * net->E))) return bad(rc);
          continue;
        }
        if ((rc = e->alloc(&net->wp[w][i], (size_t)net->E * 3 * net->kps(i)))) return bad(rc);
        if (net->x3f && (rc = e->alloc(&net->wtp[w][i], (size_t)net->E * 3 * net->wtps(i)))) return bad(rc);
      }
    if (net == &e->actor && net->E == 1 && net->width % 4 == 0 &&
        (rc = e->alloc(&net->whT, (size_t)e->T_l * net->width * net->hd)))
      return bad(rc);
  }
  {  // split-K workspaces: the largest GEMM that splits, per lane
    long long ws = 0;
    for (Net* net : {&e->actor, &e->critic})
      for (int i = 0; i < net->depth; ++i) {
        const int M = i == 0 ? net->in_dim : net->width;
        ws = std::max(ws, gemm_ws_floats(M, net->width, net->E, gemm_splits(M, net->width, e->B, net->E)));
        if (e->planes) {
          ws = std::max(ws, gemm_x3p_ws_floats(M, net->width, (int)net->krows, net->E, true));  // weight grad
          for (int rows : {e->B, net == &e->actor ? (int)(net->krows + e->B) : e->B}) {  // data grad, forward
            ws = std::max(ws, gemm_x3p_ws_floats(rows, net->width, (int)(i == 0 ? net->xld : net->ald), net->E, false));
            ws = std::max(ws, gemm_x3f_ws_floats(rows, net->width,
                                                 (int)(i == 0 ? align_up(net->in_dim, 64) : net->ald), net->E));
          }
        }
      }
    for (float*& w : e->ws_lane)
      if ((rc = e->alloc(&w, (size_t)std::max(ws, 1LL)))) return bad(rc);
    if (e->planes && e->defer_finish())  // the deferred weight-grad finishes' slabs, per layer (Net::fin_sink);
      for (Net* net : {&e->actor, &e->critic})  // not with MTSAC_DEFER_FINISH=0 (sharded runs never use them either,
                                                 // but sharding is set after create)
        for (int i = 0; i < net->depth; ++i) {
          const long long w = gemm_x3p_ws_floats(i == 0 ? net->in_dim : net->width, net->width, (int)net->krows,
                                                 net->E, true);
          if (w > 0 && (rc = e->alloc(&net->ws_wg[i], (size_t)w))) return bad(rc);
        }
    for (int*& c : e->cnt_lane)
      if ((rc = e->alloc(&c, (size_t)GEMM_X3F_CNT))) return bad(rc);
  }
  for (Net* net : {&e->actor, &e->critic})
    for (int i = 0; i < net->depth; ++i)
      if (net->bfrag[i]) net->bfrag[i] = e->frag_probe(*net, i);

  const int B = e->B;
  if ((rc = e->alloc(&e->store, (size_t)c.capacity * e->T_l * e->R))) return bad(rc);
  if ((rc = e->alloc(&e->buf_size, 1))) return bad(rc);
  if ((rc = e->alloc(&e->rng, 1))) return bad(rc);
  if ((rc = e->alloc(&e->jump, 65 * 4))) return bad(rc);
  if ((rc = e->alloc(&e->idx, e->n))) return bad(rc);
  if ((rc = e->alloc(&e->rmin, e->T_l))) return bad(rc);
  if ((rc = e->alloc(&e->rmax, e->T_l))) return bad(rc);
  e->Ma = (int)(e->actor.krows + B);
  for (auto& q : e->inset) {
    if ((rc = e->alloc(&q.xa, (size_t)e->Ma * e->ld_a))) return bad(rc);  // [s | pad | s'], pad rows stay 0
    if ((rc = e->alloc(&q.task, B)) || (rc = e->alloc(&q.counts, e->T_l)) || (rc = e->alloc(&q.rows, (size_t)e->T_l * B)))
      return bad(rc);
  }
  e->xa = e->inset[0].xa;
  e->xan = e->xa + e->actor.krows * e->ld_a;
  e->task = e->inset[0].task;
  e->counts = e->inset[0].counts;
  e->rows = e->inset[0].rows;
  {
    std::vector<int> sc(e->T_l, e->n), sr((size_t)e->T_l * B, 0);
    for (int t = 0; t < e->T_l; ++t)
      for (int i = 0; i < e->n; ++i) sr[(size_t)t * B + i] = i * e->T_l + t;
    if ((rc = e->alloc(&e->s_counts, e->T_l)) || (rc = e->alloc(&e->s_rows, (size_t)e->T_l * B))) return bad(rc);
    if (hipMemcpy(e->s_counts, sc.data(), sizeof(int) * sc.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->s_rows, sr.data(), sizeof(int) * sr.size(), hipMemcpyHostToDevice) != hipSuccess)
      return bad(fail(-5, "row lists"));
  }
  if ((rc = e->alloc(&e->xc, (size_t)B * e->ld_c))) return bad(rc);
  if ((rc = e->alloc(&e->xcn, (size_t)B * e->ld_c))) return bad(rc);
  if ((rc = e->alloc(&e->xcp, (size_t)B * e->ld_c))) return bad(rc);
  for (float** p : {&e->rew, &e->done, &e->tw, &e->logpi_n, &e->logpi, &e->y, &e->row_a, &e->row_b, &e->row_c,
                    &e->alpha_w, &e->u_done, &e->u_rew})
    if ((rc = e->alloc(p, B))) return bad(rc);

  if ((rc = e->alloc(&e->u_obs, (size_t)B * e->D))) return bad(rc);
  if ((rc = e->alloc(&e->u_nobs, (size_t)B * e->D))) return bad(rc);
  if ((rc = e->alloc(&e->u_act, (size_t)B * e->A))) return bad(rc);
  if ((rc = e->alloc(&e->eps_n, (size_t)B * e->A))) return bad(rc);
  if ((rc = e->alloc(&e->eps_c, (size_t)B * e->A))) return bad(rc);
  for (int i = 0; i < c.actor_depth; ++i) {
    if ((rc = e->alloc(&e->ha[i], (size_t)e->Ma * c.actor_width))) return bad(rc);
    e->han[i] = e->ha[i] + e->actor.krows * c.actor_width;
    if ((rc = e->alloc(&e->dza[i], (size_t)B * c.actor_width))) return bad(rc);
  }
  for (int i = 0; i < c.critic_depth; ++i)
    for (float** p : {&e->hc[i], &e->hct[i], &e->dzc[i]})
      if ((rc = e->alloc(p, (size_t)c.num_critics * B * c.critic_width))) return bad(rc);
  if (e->planes) {
    for (Net* net : {&e->actor, &e->critic}) {
      const bool cr = net == &e->critic;
      const size_t np = (size_t)net->E * 3 * net->aps();
      for (int i = 0; i + 1 < net->depth; ++i) {
        if ((rc = e->alloc(cr ? &e->hcp[i] : &e->hap[i], np))) return bad(rc);
        if (!cr) e->hap_s2[i] = e->hap[i] + net->krows * net->ald;
        if (cr && (rc = e->alloc(&e->hctp[i], np))) return bad(rc);
      }
      // dz[0] planes (in_wgrad_planes): the input layer's weight grad (K = B, M = in_dim) on k-major
      // planes; else it runs on the on-the-fly split kernel from the fp32 dz[0]
      const int d0 = e->in_wgrad_planes ? 0 : 1;
      for (int i = d0; i < net->depth; ++i)
        if ((rc = e->alloc(cr ? &e->dzcp[i] : &e->dzap[i], np))) return bad(rc);
      const long long chunks = std::max<long long>({(long long)COLSUM_CHUNKS, gemm_x3f_max_row_tiles(e->B),
                                                    head_backward_chunks(e->T_l)});
      for (int i = d0; i < net->depth; ++i)
        if ((rc = e->alloc(&net->dbp[i], (size_t)(net->E * chunks * net->width)))) return bad(rc);
    }
    {
      const float* xs[5] = {e->xa, e->xan, e->xc, e->xcn, e->xcp};
      for (int k = 0; k < 5; ++k) {
        const Net& net = k < 2 ? e->actor : e->critic;
        if (k == 1) continue;  // s' rows are part of xa's planes (the merged actor forward)
        e->inp[k].x = xs[k];
        if ((rc = e->alloc(&e->inp[k].p, (size_t)3 * net.arows * net.xld))) return bad(rc);
      }
      e->inset[0].xap = e->inp[0].p;  // the second input set's planes (cross-step pipelining)
      if ((rc = e->alloc(&e->inset[1].xap, (size_t)3 * e->actor.arows * e->actor.xld))) return bad(rc);
    }
    const int wmax = std::max(c.actor_width, c.critic_width);
    if ((rc = e->alloc(&e->cs_part, (size_t)std::max(1, c.num_critics) * COLSUM_CHUNKS * wmax))) return bad(rc);
  }
  if ((rc = e->alloc(&e->dq, (size_t)c.num_critics * B))) return bad(rc);
  if ((rc = e->alloc(&e->cache, (size_t)B * 5 * e->A))) return bad(rc);
  if ((rc = e->alloc(&e->dout_a, (size_t)B * 2 * e->A))) return bad(rc);
  if ((rc = e->alloc(&e->partials, 2 * PART))) return bad(rc);  // elementwise + tiled update
  if ((rc = e->alloc(&e->zparts, 256)) || (rc = e->alloc(&e->zscr, 2048))) return bad(rc);  // sharded optimizer
  if ((rc = e->alloc(&e->pn, 4))) return bad(rc);
  if ((rc = e->alloc(&e->log_alpha, e->T_g))) return bad(rc);
  if ((rc = e->alloc(&e->la_m, e->T_g))) return bad(rc);
  if ((rc = e->alloc(&e->la_v, e->T_g))) return bad(rc);
  if ((rc = e->alloc(&e->alpha_tmp, e->T_g))) return bad(rc);
  if ((rc = e->alloc(&e->sc_alpha, 1))) return bad(rc);
  if ((rc = e->alloc(&e->logs, MTSAC_NUM_LOGS))) return bad(rc);
  if ((rc = e->alloc(&e->counter, 1))) return bad(rc);
  if ((rc = e->alloc(&e->err, 2))) return bad(rc);  // [0] batch check, [1] self-check
  // rollout workspace
  const int rm = e->roll_max;
  if ((rc = e->alloc(&e->r_obs, (size_t)rm * e->D))) return bad(rc);
  if ((rc = e->alloc(&e->r_x, (size_t)rm * e->ld_a))) return bad(rc);
  if ((rc = e->alloc(&e->r_eps, (size_t)rm * e->A))) return bad(rc);
  if ((rc = e->alloc(&e->r_act, (size_t)rm * e->A))) return bad(rc);
  if ((rc = e->alloc(&e->r_lp, rm))) return bad(rc);
  if ((rc = e->alloc(&e->r_dummy, (size_t)rm * (e->ld_c + 4)))) return bad(rc);
  if ((rc = e->alloc(&e->r_task, rm))) return bad(rc);
  for (int i = 0; i < c.actor_depth; ++i)
    if ((rc = e->alloc(&e->r_h[i], (size_t)rm * c.actor_width))) return bad(rc);

  unsigned long long jt[65 * 4];
  pcg_jump_table(jt);
  if (hipMemcpy(e->jump, jt, sizeof(jt), hipMemcpyHostToDevice) != hipSuccess) return bad(fail(-5, "jump table"));
  std::vector<float> la(e->T_g, std::log(c.initial_temperature));
  if (hipMemcpy(e->log_alpha, la.data(), sizeof(float) * e->T_g, hipMemcpyHostToDevice) != hipSuccess)
    return bad(fail(-5, "log_alpha"));
  {
    std::vector<double> mn(e->T_l, INFINITY), mx(e->T_l, -INFINITY);  // buffers.py:266-267
    if (c.normalize_rewards == 2) {  // no completed episode yet: denominator 1 (buffers.py:417-418)
      std::fill(mn.begin(), mn.end(), 0.0);
      std::fill(mx.begin(), mx.end(), 1.0);
    }
    if (hipMemcpy(e->rmin, mn.data(), sizeof(double) * e->T_l, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->rmax, mx.data(), sizeof(double) * e->T_l, hipMemcpyHostToDevice) != hipSuccess)
      return bad(fail(-5, "reward stats"));
  }
  if (hipHostMalloc((void**)&e->stage_h, sizeof(float) * mtsac_engine::NSTAGE * e->T_l * e->R) != hipSuccess)
    return bad(fail(-12, "pinned staging"));
  for (hipEvent_t& x : e->stage_ev)
    if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) return bad(fail(-5, "event"));
  if (hipEventCreateWithFlags(&e->add_ev, hipEventDisableTiming) != hipSuccess) return bad(fail(-5, "event"));
  for (int k = 0; k < mtsac_engine::NSTAGE; ++k)
    if (hipEventCreateWithFlags(&e->dstage_ev[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->dpack_ev[k], hipEventDisableTiming) != hipSuccess)
      return bad(fail(-5, "event"));
  if ((rc = e->alloc(&e->dstage, (size_t)mtsac_engine::NSTAGE * e->T_l * e->R))) return bad(rc);
  for (int k = 0; k < 2; ++k)
    if (hipEventCreateWithFlags(&e->ev_ap[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_tail[k], hipEventDisableTiming) != hipSuccess)
      return bad(fail(-5, "event"));
  // the zero fills of alloc() run on the null stream, which the engine's non-blocking streams do not
  // wait for: finish them before any engine work can touch the buffers
  if (hipDeviceSynchronize() != hipSuccess) return bad(fail(-5, "device synchronize"));
  *out = e;
  return 0;
}

void mtsac_destroy(mtsac_engine* h) { delete h; }

static Net* net_of(mtsac_engine* h, int which, float** buf) {
  switch (which) {
    case MTSAC_ACTOR: *buf = h->actor.p; return &h->actor;
    case MTSAC_CRITIC: *buf = h->critic.p; return &h->critic;
    case MTSAC_CRITIC_TARGET: *buf = h->critic.tgt; return &h->critic;
    case MTSAC_ACTOR_ADAM_MU: *buf = h->actor.m; return &h->actor;
    case MTSAC_ACTOR_ADAM_NU: *buf = h->actor.v; return &h->actor;
    case MTSAC_CRITIC_ADAM_MU: *buf = h->critic.m; return &h->critic;
    case MTSAC_CRITIC_ADAM_NU: *buf = h->critic.v; return &h->critic;
    default: return nullptr;
  }
}

static float* alpha_buf(mtsac_engine* h, int which) {
  switch (which) {
    case MTSAC_LOG_ALPHA_PARAMS: return h->log_alpha;
    case MTSAC_ALPHA_ADAM_MU: return h->la_m;
    case MTSAC_ALPHA_ADAM_NU: return h->la_v;
    default: return nullptr;
  }
}

int64_t mtsac_param_count(const mtsac_engine* hc, int which) {
  auto* h = const_cast<mtsac_engine*>(hc);
  if (!h) return fail(-22, "null engine");
  if (alpha_buf(h, which)) return h->T_g;
  float* b = nullptr;
  Net* net = net_of(h, which, &b);
  if (!net) return fail(-22, "unknown tensor id");
  return net->n_params;
}

static int copy_params(mtsac_engine* h, int which, float* host, int64_t n, bool to_device) {
  if (!h || !host) return fail(-22, "null argument");
  if (float* ab = alpha_buf(h, which)) {
    if (n != h->T_g) return fail(-22, "size mismatch");
    HIP_TRY(hipStreamSynchronize(h->st));
    HIP_TRY(to_device ? hipMemcpy(ab, host, sizeof(float) * n, hipMemcpyDefault)
                      : hipMemcpy(host, ab, sizeof(float) * n, hipMemcpyDefault));
    return 0;
  }
  float* buf = nullptr;
  Net* net = net_of(h, which, &buf);
  if (!net) return fail(-22, "unknown tensor id");
  if (n != net->n_params) return fail(-22, "size mismatch: expected " + std::to_string(net->n_params));
  HIP_TRY(hipStreamSynchronize(h->st));
  long long o = 0;
  for (auto& lf : net->leaves) {
    if (to_device)
      HIP_TRY(hipMemcpy(buf + lf.first, host + o, sizeof(float) * lf.second, hipMemcpyDefault));
    else
      HIP_TRY(hipMemcpy(host + o, buf + lf.first, sizeof(float) * lf.second, hipMemcpyDefault));
    o += lf.second;
  }
  if (to_device && (buf == net->p || buf == net->tgt)) {
    if (h->h2) weights_record(buf, net->trunk_off, net->n_flat, h->w_rec(*net, buf == net->p ? 0 : 1).d, h->st);
    h->refresh_wt(*net, buf, buf == net->p ? 0 : 1, h->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(h->st));
  }
  return 0;
}

int mtsac_set_params(mtsac_engine* h, int which, const float* src, int64_t n) {
  return copy_params(h, which, const_cast<float*>(src), n, true);
}
int mtsac_get_params(mtsac_engine* h, int which, float* dst, int64_t n) { return copy_params(h, which, dst, n, false); }

static OptScalars* sc_of(mtsac_engine* h, int which) {
  return which == 0 ? h->actor.sc : which == 1 ? h->critic.sc : which == 2 ? h->sc_alpha : nullptr;
}
int mtsac_set_adam_count(mtsac_engine* h, int which, int32_t count) {
  if (!h) return fail(-22, "null engine");
  OptScalars* s = sc_of(h, which);
  if (!s) return fail(-22, "which must be 0 (actor), 1 (critic) or 2 (alpha)");
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(&s->count, &count, sizeof(int), hipMemcpyHostToDevice));
  return 0;
}
int mtsac_get_adam_count(mtsac_engine* h, int which, int32_t* count) {
  if (!h || !count) return fail(-22, "null argument");
  OptScalars* s = sc_of(h, which);
  if (!s) return fail(-22, "which must be 0 (actor), 1 (critic) or 2 (alpha)");
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(count, &s->count, sizeof(int), hipMemcpyDeviceToHost));
  return 0;
}

// ---------------------------------------------------------------- buffer
static int upload_size(mtsac_engine* h) {
  long long sz = h->h_full ? h->cfg.capacity : h->h_pos;
  HIP_TRY(hipMemcpyAsync(h->buf_size, &sz, sizeof(sz), hipMemcpyHostToDevice, h->st));
  HIP_TRY(hipStreamSynchronize(h->st));
  return 0;
}

// true for device (hipMalloc) memory; host pageable / pinned / unknown pointers are host
static bool on_device(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

// n floats from a caller pointer (host or device) into host memory
static int fetch(float* dst, const float* src, size_t n) {
  if (n == 0) return 0;
  HIP_TRY(hipMemcpy(dst, src, sizeof(float) * n, hipMemcpyDefault));
  return 0;
}

static int write_slots(mtsac_engine* h, int64_t s0, int64_t ns, const float* obs, const float* nobs, const float* act,
                       const float* rew, const float* done) {
  const int T = h->T_l, D = h->D, A = h->A, R = h->R;
  const size_t rows = (size_t)ns * T;
  std::vector<float> o(rows * D), no(rows * D), a(rows * A), r(rows), d(rows);
  int rc = 0;
  if ((rc = fetch(o.data(), obs, o.size())) || (rc = fetch(no.data(), nobs, no.size())) ||
      (rc = fetch(a.data(), act, a.size())) || (rc = fetch(r.data(), rew, rows)) || (rc = fetch(d.data(), done, rows)))
    return rc;
  std::vector<float> rec(rows * R, 0.0f);
  for (size_t row = 0; row < rows; ++row) {
    float* x = &rec[row * R];
    std::memcpy(x, &o[row * D], sizeof(float) * D);
    std::memcpy(x + D, &a[row * A], sizeof(float) * A);
    x[D + A] = r[row];
    x[D + A + 1] = d[row];
    std::memcpy(x + D + A + 2, &no[row * D], sizeof(float) * D);
  }
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(h->store + (size_t)s0 * T * R, rec.data(), sizeof(float) * rec.size(), hipMemcpyHostToDevice));
  if (h->bufmax) {  // split2h: the stored rows' max |obs|, |action|, |next_obs| only grows
    float m = 0.f, cur = 0.f;
    for (float v : o) m = std::max(m, std::fabs(v));
    for (float v : no) m = std::max(m, std::fabs(v));
    for (float v : a) m = std::max(m, std::fabs(v));
    HIP_TRY(hipMemcpy(&cur, h->bufmax, sizeof(float), hipMemcpyDeviceToHost));
    if (m > cur) HIP_TRY(hipMemcpy(h->bufmax, &m, sizeof(float), hipMemcpyHostToDevice));
  }
  return 0;
}

// add (buffers.py:426-474 + _advance_position :337-343) without blocking the host: the slot is
// packed into a pinned staging slot (host pointers) or by a kernel (device pointers) and copied
// / committed on the engine stream, so it lands after every update issued before it and before
// every update issued after it; pos / full advance on the host, the sampled range and the
// reward min / max on the device.
int mtsac_buffer_add(mtsac_engine* h, const float* obs, const float* next_obs, const float* actions,
                     const float* rewards, const float* dones) {
  return mtsac_buffer_add_stream(h, obs, next_obs, actions, rewards, dones, nullptr);
}

int mtsac_buffer_add_stream(mtsac_engine* h, const float* obs, const float* next_obs, const float* actions,
                            const float* rewards, const float* dones, void* producer_stream) {
  if (!h || !obs || !next_obs || !actions || !rewards || !dones) return fail(-22, "null argument");
  const int T = h->T_l, D = h->D, A = h->A, R = h->R;
  const int ndev = (int)on_device(obs) + (int)on_device(next_obs) + (int)on_device(actions) +
                   (int)on_device(rewards) + (int)on_device(dones);
  if (ndev != 0 && ndev != 5) return fail(-22, "buffer_add: pass all five arrays in host memory or all in device memory");
  float* slot = h->store + (size_t)h->h_pos * T * R;
  if (ndev == 5) {
    // Device arrays: the pack into a staging record runs on the side stream after the producer's
    // queued work (and after the engine stream has copied that record's previous contents out);
    // the producer stream waits for the pack only -- not for the updates queued on the engine
    // stream -- before anything it issues next (a caching allocator hands a freed block to the next
    // allocation on that stream), so the caller may drop or overwrite the arrays as soon as this
    // returns.  The engine stream then copies the record into the store slot in update order.
    hipStream_t prod = static_cast<hipStream_t>(producer_stream);
    const int k = h->dstage_next;
    h->dstage_next = (k + 1) % mtsac_engine::NSTAGE;
    float* rec = h->dstage + (size_t)k * T * R;
    HIP_TRY(hipEventRecord(h->add_ev, prod));
    HIP_TRY(hipStreamWaitEvent(h->sa, h->add_ev, 0));
    HIP_TRY(hipStreamWaitEvent(h->sa, h->dstage_ev[k], 0));  // the record's previous copy-out
    buffer_pack_slot(rec, T, R, D, A, obs, next_obs, actions, rewards, dones, h->sa);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->dpack_ev[k], h->sa));
    HIP_TRY(hipStreamWaitEvent(prod, h->dpack_ev[k], 0));
    HIP_TRY(hipStreamWaitEvent(h->st, h->dpack_ev[k], 0));
    HIP_TRY(hipMemcpyAsync(slot, rec, sizeof(float) * T * R, hipMemcpyDeviceToDevice, h->st));
    HIP_TRY(hipEventRecord(h->dstage_ev[k], h->st));
  } else {
    const int k = h->stage_next;
    h->stage_next = (k + 1) % mtsac_engine::NSTAGE;
    HIP_TRY(hipEventSynchronize(h->stage_ev[k]));  // that staging slot's previous copy is done
    float* rec = h->stage_h + (size_t)k * T * R;
    for (int t = 0; t < T; ++t) {
      float* x = rec + (size_t)t * R;
      std::memcpy(x, obs + (size_t)t * D, sizeof(float) * D);
      std::memcpy(x + D, actions + (size_t)t * A, sizeof(float) * A);
      x[D + A] = rewards[t];
      x[D + A + 1] = dones[t];
      std::memcpy(x + D + A + 2, next_obs + (size_t)t * D, sizeof(float) * D);
      for (int c = 2 * D + A + 2; c < R; ++c) x[c] = 0.f;
    }
    HIP_TRY(hipMemcpyAsync(slot, rec, sizeof(float) * T * R, hipMemcpyHostToDevice, h->st));
    HIP_TRY(hipEventRecord(h->stage_ev[k], h->st));
  }
  const long long np = h->h_pos + 1;
  if (np >= h->cfg.capacity) h->h_full = 1;
  h->h_pos = np % h->cfg.capacity;
  buffer_commit_slot(slot, T, R, D + A, h->cfg.normalize_rewards == 1 ? h->rmin : nullptr, h->rmax, h->buf_size,
                     h->h_full ? h->cfg.capacity : h->h_pos, h->st, D, h->bufmax);
  HIP_TRY(hipGetLastError());
  return 0;
}

int mtsac_buffer_write(mtsac_engine* h, int64_t s0, int64_t ns, const float* obs, const float* next_obs,
                       const float* actions, const float* rewards, const float* dones) {
  if (!h || !obs || !next_obs || !actions || !rewards || !dones) return fail(-22, "null argument");
  if (s0 < 0 || ns < 0 || s0 + ns > h->cfg.capacity) return fail(-22, "slot range out of bounds");
  const int64_t chunk = 4096;
  for (int64_t s = 0; s < ns; s += chunk) {
    const int64_t k = std::min(chunk, ns - s);
    const size_t row = (size_t)s * h->T_l;
    int rc = write_slots(h, s0 + s, k, obs + row * h->D, next_obs + row * h->D, actions + row * h->A, rewards + row,
                         dones + row);
    if (rc) return rc;
  }
  return 0;
}

int mtsac_buffer_read(mtsac_engine* h, int64_t s0, int64_t ns, float* obs, float* next_obs, float* actions,
                      float* rewards, float* dones) {
  if (!h) return fail(-22, "null engine");
  if (s0 < 0 || ns < 0 || s0 + ns > h->cfg.capacity) return fail(-22, "slot range out of bounds");
  const int T = h->T_l, D = h->D, A = h->A, R = h->R;
  const size_t rows = (size_t)ns * T;
  std::vector<float> rec(rows * R);
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(rec.data(), h->store + (size_t)s0 * T * R, sizeof(float) * rec.size(), hipMemcpyDeviceToHost));
  std::vector<float> o(rows * D), no(rows * D), a(rows * A), r(rows), d(rows);
  for (size_t row = 0; row < rows; ++row) {
    const float* x = &rec[row * R];
    std::memcpy(&o[row * D], x, sizeof(float) * D);
    std::memcpy(&a[row * A], x + D, sizeof(float) * A);
    r[row] = x[D + A];
    d[row] = x[D + A + 1];
    std::memcpy(&no[row * D], x + D + A + 2, sizeof(float) * D);
  }
  // the caller's pointers may be host or device memory
  if (obs) HIP_TRY(hipMemcpy(obs, o.data(), sizeof(float) * o.size(), hipMemcpyDefault));
  if (next_obs) HIP_TRY(hipMemcpy(next_obs, no.data(), sizeof(float) * no.size(), hipMemcpyDefault));
  if (actions) HIP_TRY(hipMemcpy(actions, a.data(), sizeof(float) * a.size(), hipMemcpyDefault));
  if (rewards) HIP_TRY(hipMemcpy(rewards, r.data(), sizeof(float) * rows, hipMemcpyDefault));
  if (dones) HIP_TRY(hipMemcpy(dones, d.data(), sizeof(float) * rows, hipMemcpyDefault));
  return 0;
}

int mtsac_buffer_fill_synthetic(mtsac_engine* h, uint64_t seed) {
  if (!h) return fail(-22, "null engine");
  fill_synthetic(h->store, h->cfg.capacity, h->T_l, h->R, h->D, h->A, h->T_g, h->cfg.task_begin, seed, h->st,
                 h->bufmax);
  HIP_TRY(hipGetLastError());
  h->h_pos = 0;
  h->h_full = 1;
  return upload_size(h);
}

int mtsac_buffer_set_state(mtsac_engine* h, int64_t pos, int32_t full) {
  if (!h) return fail(-22, "null engine");
  if (pos < 0 || pos >= h->cfg.capacity) return fail(-22, "pos out of range");
  h->h_pos = pos;
  h->h_full = full ? 1 : 0;
  return upload_size(h);
}

int mtsac_buffer_get_state(mtsac_engine* h, int64_t* pos, int32_t* full) {
  if (!h || !pos || !full) return fail(-22, "null argument");
  *pos = h->h_pos;
  *full = h->h_full;
  return 0;
}

int mtsac_buffer_set_reward_stats(mtsac_engine* h, const double* mn, const double* mx) {
  if (!h || !mn || !mx) return fail(-22, "null argument");
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(h->rmin, mn, sizeof(double) * h->T_l, hipMemcpyDefault));
  HIP_TRY(hipMemcpy(h->rmax, mx, sizeof(double) * h->T_l, hipMemcpyDefault));
  return 0;
}

int mtsac_buffer_get_reward_stats(mtsac_engine* h, double* mn, double* mx) {
  if (!h || !mn || !mx) return fail(-22, "null argument");
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(mn, h->rmin, sizeof(double) * h->T_l, hipMemcpyDefault));
  HIP_TRY(hipMemcpy(mx, h->rmax, sizeof(double) * h->T_l, hipMemcpyDefault));
  return 0;
}

int mtsac_rng_set(mtsac_engine* h, uint64_t shi, uint64_t slo, uint64_t ihi, uint64_t ilo, int32_t has32, uint32_t u) {
  if (!h) return fail(-22, "null engine");
  PcgDev s{shi, slo, ihi, ilo, has32 ? 1 : 0, u};
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(h->rng, &s, sizeof(s), hipMemcpyHostToDevice));
  return 0;
}

int mtsac_rng_get(mtsac_engine* h, uint64_t* shi, uint64_t* slo, uint64_t* ihi, uint64_t* ilo, int32_t* has32,
                  uint32_t* u) {
  if (!h || !shi || !slo || !ihi || !ilo || !has32 || !u) return fail(-22, "null argument");
  PcgDev s{};
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(&s, h->rng, sizeof(s), hipMemcpyDeviceToHost));
  *shi = s.state_hi;
  *slo = s.state_lo;
  *ihi = s.inc_hi;
  *ilo = s.inc_lo;
  *has32 = s.has_uint32;
  *u = s.uinteger;
  return 0;
}

int mtsac_sample(mtsac_engine* h, int64_t* indices, float* obs, float* actions, float* next_obs, float* dones,
                 float* rewards) {
  if (!h) return fail(-22, "null engine");
  replay_indices(h->rng, h->jump, h->buf_size, h->n, h->idx, h->st);
  GatherParams gp = h->gather_params();
  replay_gather(gp, h->st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(h->st));
  const int B = h->B, D = h->D, A = h->A;
  if (indices) {
    std::vector<int> tmp(h->n);
    HIP_TRY(hipMemcpy(tmp.data(), h->idx, sizeof(int) * h->n, hipMemcpyDeviceToHost));
    std::vector<int64_t> wide(tmp.begin(), tmp.end());
    HIP_TRY(hipMemcpy(indices, wide.data(), sizeof(int64_t) * h->n, hipMemcpyDefault));
  }
  if (obs) HIP_TRY(hipMemcpy2D(obs, sizeof(float) * D, h->xa, sizeof(float) * h->ld_a, sizeof(float) * D, B,
                               hipMemcpyDefault));
  if (next_obs) HIP_TRY(hipMemcpy2D(next_obs, sizeof(float) * D, h->xan, sizeof(float) * h->ld_a, sizeof(float) * D,
                                    B, hipMemcpyDefault));
  if (actions) HIP_TRY(hipMemcpy2D(actions, sizeof(float) * A, h->xc, sizeof(float) * h->ld_c, sizeof(float) * A, B,
                                   hipMemcpyDefault));
  if (dones) HIP_TRY(hipMemcpy(dones, h->done, sizeof(float) * B, hipMemcpyDefault));
  if (rewards) HIP_TRY(hipMemcpy(rewards, h->rew, sizeof(float) * B, hipMemcpyDefault));
  return h->check_err();
}

// ---------------------------------------------------------------- update
int mtsac_update(mtsac_engine* h, const mtsac_batch* b, const float* eps_next, const float* eps_cur) {
  if (!h) return fail(-22, "null engine");
  if (int rc = h->geo_guard()) return rc;
  if ((eps_next == nullptr) != (eps_cur == nullptr)) return fail(-22, "inject both eps_next and eps_cur or neither");
  const int B = h->B, D = h->D, A = h->A;
  if (b) {
    if (!b->observations || !b->actions || !b->next_observations || !b->dones || !b->rewards)
      return fail(-22, "incomplete batch");
    HIP_TRY(hipMemcpyAsync(h->u_obs, b->observations, sizeof(float) * B * D, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_nobs, b->next_observations, sizeof(float) * B * D, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_act, b->actions, sizeof(float) * B * A, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_done, b->dones, sizeof(float) * B, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_rew, b->rewards, sizeof(float) * B, hipMemcpyDefault, h->st));
  }
  if (eps_next) {
    HIP_TRY(hipMemcpyAsync(h->eps_n, eps_next, sizeof(float) * B * A, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->eps_c, eps_cur, sizeof(float) * B * A, hipMemcpyDefault, h->st));
  }
  h->tl_next = 0;
  h->step(b == nullptr, eps_next == nullptr);
  HIP_TRY(hipGetLastError());
  if (b || eps_next) HIP_TRY(hipStreamSynchronize(h->st));  // borrowed host pointers
  return 0;
}

// ---------------------------------------------------------------- gradient-conflict metrics
static int task_grad_ready(mtsac_engine* h, int which) {
  if (!h) return fail(-22, "null engine");
  if (which != 0 && which != 1) return fail(-22, "which: 0 critic, 1 actor");
  if (!h->tg[which]) return fail(-22, "no per-task gradients yet (mtsac_task_gradients)");
  return 0;
}

int mtsac_task_gradients(mtsac_engine* h, const mtsac_batch* b, const float* eps_next, const float* eps_cur) {
  if (!h) return fail(-22, "null engine");
  if (int rc = h->geo_guard()) return rc;
  if (h->T_l != h->T_g) return fail(-95, "per-task gradients need every task on one engine (unsharded)");
  if ((eps_next == nullptr) != (eps_cur == nullptr)) return fail(-22, "inject both eps_next and eps_cur or neither");
  int rc = h->ensure_task_grad_buffers();
  if (rc) return rc;
  const int B = h->B, D = h->D, A = h->A;
  if (b) {
    if (!b->observations || !b->actions || !b->next_observations || !b->dones || !b->rewards)
      return fail(-22, "incomplete batch");
    HIP_TRY(hipMemcpyAsync(h->u_obs, b->observations, sizeof(float) * B * D, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_nobs, b->next_observations, sizeof(float) * B * D, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_act, b->actions, sizeof(float) * B * A, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_done, b->dones, sizeof(float) * B, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->u_rew, b->rewards, sizeof(float) * B, hipMemcpyDefault, h->st));
  }
  if (eps_next) {
    HIP_TRY(hipMemcpyAsync(h->eps_n, eps_next, sizeof(float) * B * A, hipMemcpyDefault, h->st));
    HIP_TRY(hipMemcpyAsync(h->eps_c, eps_cur, sizeof(float) * B * A, hipMemcpyDefault, h->st));
  }
  const bool timing = h->timing;
  h->timing = false;
  h->task_grads(b == nullptr, eps_next == nullptr);
  h->timing = timing;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(h->st));
  int e = 0;
  HIP_TRY(hipMemcpy(&e, h->err, sizeof(int), hipMemcpyDeviceToHost));
  if (e) {
    int z = 0;
    HIP_TRY(hipMemcpy(h->err, &z, sizeof(int), hipMemcpyHostToDevice));
    return fail(-22, "batch rows must be interleaved i*T + t with exact one-hot task ids (as the buffer samples)");
  }
  return 0;
}

int64_t mtsac_task_gradient_size(const mtsac_engine* h, int which) {
  if (!h || (which != 0 && which != 1)) return -22;
  return which == 0 ? h->critic.n_params : h->actor.n_params;
}

static int copy_task_grads(mtsac_engine* h, int which, float* host, int64_t n, bool to_device) {
  if (!h) return fail(-22, "null engine");
  if (to_device && !h->tg[which]) {
    int rc = h->ensure_task_grad_buffers();
    if (rc) return rc;
  }
  int rc = task_grad_ready(h, which);
  if (rc) return rc;
  if (!host || n != (int64_t)h->T_l * h->tgP[which]) return fail(-22, "size must be T * P");
  HIP_TRY(hipStreamSynchronize(h->st));
  if (to_device) HIP_TRY(hipMemcpy(h->tg[which], host, sizeof(float) * n, hipMemcpyDefault));
  else HIP_TRY(hipMemcpy(host, h->tg[which], sizeof(float) * n, hipMemcpyDefault));
  return 0;
}

int mtsac_get_task_gradients(mtsac_engine* h, int which, float* dst, int64_t n) {
  return copy_task_grads(h, which, dst, n, false);
}

int mtsac_set_task_gradients(mtsac_engine* h, int which, const float* src, int64_t n) {
  if (h && h->T_l != h->T_g) return fail(-95, "per-task gradients need every task on one engine (unsharded)");
  return copy_task_grads(h, which, const_cast<float*>(src), n, true);
}

int mtsac_task_gradient_select(mtsac_engine* h, int which, const int64_t* ranks, float* values) {
  int rc = task_grad_ready(h, which);
  if (rc) return rc;
  if (!ranks || !values) return fail(-22, "null argument");
  const long long P = h->tgP[which];
  for (int k = 0; k < 2 * h->T_l; ++k)
    if (ranks[k] < 0 || ranks[k] >= P) return fail(-22, "rank out of range");
  std::vector<long long> r(ranks, ranks + 2 * h->T_l);
  task_select(h->tg[which], h->T_l, P, r.data(), values, h->sel_prefix, h->sel_rank, h->sel_hist, h->st);
  HIP_TRY(hipGetLastError());
  return 0;
}

int mtsac_task_gradient_stats(mtsac_engine* h, int which, const float* thresholds, float eps, float tau, double* gram,
                              double* l1, int64_t* counts, int64_t* near_zero) {
  int rc = task_grad_ready(h, which);
  if (rc) return rc;
  if (!thresholds || !gram || !l1 || !counts || !near_zero) return fail(-22, "null argument");
  const int T = h->T_l;
  HIP_TRY(hipMemcpyAsync(h->ps_thr, thresholds, sizeof(float) * T, hipMemcpyHostToDevice, h->st));
  task_pair_stats(h->tg[which], T, h->tgP[which], h->ps_thr, eps, tau, mtsac_engine::PS_GRID, h->ps_gram_part,
                  h->ps_l1_part, h->ps_counts, h->ps_nz, h->ps_gram, h->ps_l1, h->st);
  HIP_TRY(hipGetLastError());
  std::vector<double> g(64 * 64), l(64);
  std::vector<unsigned long long> c(4 * 64 * 64), z(64);
  HIP_TRY(hipMemcpyAsync(g.data(), h->ps_gram, sizeof(double) * g.size(), hipMemcpyDeviceToHost, h->st));
  HIP_TRY(hipMemcpyAsync(l.data(), h->ps_l1, sizeof(double) * l.size(), hipMemcpyDeviceToHost, h->st));
  HIP_TRY(hipMemcpyAsync(c.data(), h->ps_counts, sizeof(unsigned long long) * c.size(), hipMemcpyDeviceToHost, h->st));
  HIP_TRY(hipMemcpyAsync(z.data(), h->ps_nz, sizeof(unsigned long long) * z.size(), hipMemcpyDeviceToHost, h->st));
  HIP_TRY(hipStreamSynchronize(h->st));
  for (int i = 0; i < T; ++i) {
    l1[i] = l[i];
    near_zero[i] = (int64_t)z[i];
    for (int j = 0; j < T; ++j) {
      gram[i * T + j] = g[i * 64 + j];
      for (int q = 0; q < 4; ++q) counts[(long long)q * T * T + i * T + j] = (int64_t)c[(long long)q * 64 * 64 + i * 64 + j];
    }
  }
  return 0;
}

int mtsac_update_many(mtsac_engine* h, int32_t steps) {
  if (!h) return fail(-22, "null engine");
  if (int rc = h->geo_guard()) return rc;
  if (steps <= 0) return 0;
  if (!h->use_graph || h->timing || h->hook || h->chook) {  // events / host hooks need eager issue
    h->tl_next = 0;  // timing records every launch of this call
    // consecutive steps overlap (the last one joins every lane into the main stream); host hooks
    // (the bring-your-own all-reduce, which blocks the issuing thread) keep whole steps
    const bool pipe = !h->hook && !h->chook && h->pipeline_on();
    for (int s = 0; s < steps; ++s) h->step(true, true, pipe, s + 1 == steps);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (h->gexec && h->graph_timed != h->timing) {
    (void)hipGraphExecDestroy(h->gexec);
    (void)hipGraphDestroy(h->graph);
    h->gexec = nullptr;
    h->graph = nullptr;
  }
  if (!h->gexec) {
    h->tl_next = 0;
    HIP_TRY(hipGraphCreate(&h->graph, 0));
    h->build = h->graph;
    h->step(true, true);
    h->build = nullptr;
    if (!h->comm_error.empty()) {
      (void)hipGraphDestroy(h->graph);
      h->graph = nullptr;
      return h->check_err();
    }
    HIP_TRY(hipGraphInstantiate(&h->gexec, h->graph, nullptr, nullptr, 0));
    h->graph_timed = h->timing;
  }
  for (int s = 0; s < steps; ++s) HIP_TRY(hipGraphLaunch(h->gexec, h->st));
  return 0;
}

int mtsac_get_logs(mtsac_engine* h, float* logs) {
  if (!h || !logs) return fail(-22, "null argument");
  HIP_TRY(hipMemcpyAsync(logs, h->logs, sizeof(float) * MTSAC_NUM_LOGS, hipMemcpyDefault, h->st));
  HIP_TRY(hipStreamSynchronize(h->st));
  return h->check_err();
}

int mtsac_enable_graph(mtsac_engine* h, int32_t enable) {
  if (!h) return fail(-22, "null engine");
  h->use_graph = enable != 0;
  return 0;
}

int mtsac_synchronize(mtsac_engine* h) {
  if (!h) return fail(-22, "null engine");
  HIP_TRY(hipStreamSynchronize(h->st));
  return h->check_err();
}

// ---------------------------------------------------------------- rollout
static int act(mtsac_engine* h, const float* obs, int n, const float* eps, float* out, bool zero_eps) {
  if (!h || !obs || !out) return fail(-22, "null argument");
  if (n < 1 || n > h->roll_max) return fail(-22, "row count out of range");
  const int D = h->D, A = h->A;
  HIP_TRY(hipMemcpyAsync(h->r_obs, obs, sizeof(float) * n * D, hipMemcpyDefault, h->st));
  if (zero_eps)
    HIP_TRY(hipMemsetAsync(h->r_eps, 0, sizeof(float) * n * A, h->st));
  else
    HIP_TRY(hipMemcpyAsync(h->r_eps, eps, sizeof(float) * n * A, hipMemcpyDefault, h->st));
  GatherParams gp{};
  gp.T_l = h->T_l;
  gp.obs_dim = D;
  gp.act_dim = A;
  gp.T_glob = h->T_g;
  gp.task_begin = h->cfg.task_begin;
  gp.ld_a = h->ld_a;
  gp.ld_c = h->ld_c;
  gp.xa = h->r_x;
  gp.xa_next = h->r_dummy;
  gp.xc = h->r_dummy;
  gp.xc_next = h->r_dummy;
  gp.xc_pi = h->r_dummy;
  gp.rew = h->r_lp;
  gp.done = h->r_lp;
  gp.task = h->r_task;
  gp.err = h->err;
  // obs doubles as next_obs; the action / reward / done inputs are ignored scratch
  batch_scatter(gp, h->r_obs, h->r_eps, h->r_obs, h->r_lp, h->r_lp, n, h->st);
  h->trunk_forward(h->actor, h->actor.p, -1, h->r_x, h->ld_a, h->r_h, nullptr, n);
  PolicyParams pp{};
  pp.head = h->head(h->actor, h->actor.p, h->r_h[h->actor.depth - 1], n, h->r_task);
  pp.eps = h->r_eps;
  pp.A = A;
  pp.ls_min = h->cfg.log_std_min;
  pp.ls_max = h->cfg.log_std_max;
  pp.a_out = h->r_act;
  pp.ld_a_out = A;
  pp.logpi = h->r_lp;
  policy_head(pp, h->st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, h->r_act, sizeof(float) * n * A, hipMemcpyDefault, h->st));
  HIP_TRY(hipStreamSynchronize(h->st));
  return h->check_err();
}

int mtsac_eval_action(mtsac_engine* h, const float* obs, int32_t n, float* actions) {
  return act(h, obs, n, nullptr, actions, true);  // mode() = tanh(mu)
}
int mtsac_sample_action(mtsac_engine* h, const float* obs, int32_t n, const float* eps, float* actions) {
  if (!eps) return fail(-22, "eps required");
  return act(h, obs, n, eps, actions, false);
}

// ---------------------------------------------------------------- comm
int mtsac_comm_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }
int mtsac_comm_get_unique_id(void* id_out) {
  if (!id_out) return fail(-22, "null argument");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(-5, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}
int mtsac_comm_init(mtsac_engine* h, const void* unique_id, int32_t nranks, int32_t rank) {
  const char* v = getenv("MTSAC_COMM_INIT_TIMEOUT_S");
  return mtsac_comm_init_timeout(h, unique_id, nranks, rank, v ? atof(v) : 0.0);
}

// With timeout_s > 0 the communicator is created non-blocking (ncclConfig_t.blocking = 0) so that a
// peer that never joins (a dead rank, a wrong unique id) ends in an error after timeout_s instead of
// a hang: ncclCommInitRankConfig returns at once and the init is polled through
// ncclCommGetAsyncError; on timeout the half-built communicator is aborted.  Collectives on it may
// then return ncclInProgress while their connections are set up; allreduce() waits those out.
// timeout_s <= 0 keeps RCCL's blocking communicator.  Neither form is issued inside a graph capture:
// sharded runs step eagerly (bench.py), and non-blocking RCCL under capture is untested on >1 device.
int mtsac_comm_init_timeout(mtsac_engine* h, const void* unique_id, int32_t nranks, int32_t rank, double timeout_s) {
  if (!h || !unique_id) return fail(-22, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(-22, "bad rank / nranks");
  if (h->comm) return fail(-16, "communicator already initialised");
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  HIP_TRY(hipSetDevice(h->device));
  ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
  // non-blocking only when a timeout is asked for: then the init is polled and a peer that never
  // joins ends in -110; without one the communicator (and every collective on it) stays blocking
  config.blocking = timeout_s > 0 ? 0 : 1;
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, id, rank, &config);
  if (r != ncclSuccess && r != ncclInProgress)
    return fail(-5, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclResult_t a = ncclInProgress;
    r = ncclCommGetAsyncError(comm, &a);
    if (r != ncclSuccess) a = r;
    if (a == ncclSuccess) break;
    if (a != ncclInProgress) {
      (void)ncclCommAbort(comm);
      return fail(-5, std::string("ncclCommInitRank (rank ") + std::to_string(rank) + " of " +
                          std::to_string(nranks) + "): " + ncclGetErrorString(a));
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0 && dt > timeout_s) {
      (void)ncclCommAbort(comm);
      return fail(-110, "ncclCommInitRank (rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                            "): peers did not join within " + std::to_string(timeout_s) + " s");
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  h->comm = comm;
  h->nranks = nranks;
  h->rank = rank;
  if (h->gexec) {
    (void)hipGraphExecDestroy(h->gexec);
    (void)hipGraphDestroy(h->graph);
    h->gexec = nullptr;
    h->graph = nullptr;
  }
  return 0;
}

int mtsac_get_noise_state(mtsac_engine* h, uint64_t* seed, uint64_t* counter) {
  if (!h || !seed || !counter) return fail(-22, "null argument");
  unsigned long long c = 0;
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(&c, h->counter, sizeof(c), hipMemcpyDeviceToHost));
  *seed = h->cfg.noise_seed;
  *counter = c;
  return 0;
}

int mtsac_set_noise_state(mtsac_engine* h, uint64_t seed, uint64_t counter) {
  if (!h) return fail(-22, "null engine");
  unsigned long long c = counter;
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(h->counter, &c, sizeof(c), hipMemcpyHostToDevice));
  if (seed != h->cfg.noise_seed) {  // the seed is a kernel argument inside the step graph
    h->cfg.noise_seed = seed;
    if (h->gexec) {
      (void)hipGraphExecDestroy(h->gexec);
      (void)hipGraphDestroy(h->graph);
      h->gexec = nullptr;
      h->graph = nullptr;
    }
  }
  return 0;
}

int mtsac_comm_nranks(mtsac_engine* h, int32_t* nranks) {
  if (!h || !nranks) return fail(-22, "null argument");
  int n = 1;
  if (h->comm) {
    ncclResult_t r = ncclCommCount(h->comm, &n);
    if (r != ncclSuccess) return fail(-5, std::string("ncclCommCount: ") + ncclGetErrorString(r));
  }
  *nranks = n;
  return 0;
}

int mtsac_set_allreduce_hook(mtsac_engine* h, mtsac_allreduce_fn fn, void* user) {
  if (!h) return fail(-22, "null engine");
  h->hook = fn;
  h->hook_user = user;
  if (fn) h->chook = nullptr;
  return 0;
}

int mtsac_set_collective_hook(mtsac_engine* h, mtsac_collective_fn fn, void* user, int32_t rank, int32_t world) {
  if (!h) return fail(-22, "null engine");
  if (fn && (world < 1 || rank < 0 || rank >= world)) return fail(-22, "bad rank / world");
  h->chook = fn;
  h->chook_user = user;
  h->hook_rank = fn ? rank : 0;
  h->hook_world = fn ? world : 1;
  if (fn) h->hook = nullptr;
  return 0;
}

int mtsac_set_sharded_optimizer(mtsac_engine* h, int32_t on) {
  if (!h) return fail(-22, "null engine");
  const int want = on ? 1 : 0;
  if (want == h->zero_req) return 0;
  HIP_TRY(hipStreamSynchronize(h->st));
  h->zero_req = want;
  if (h->gexec) {  // the captured step holds the other optimizer form (bucket ops, optimize_zero)
    (void)hipGraphExecDestroy(h->gexec);
    (void)hipGraphDestroy(h->graph);
    h->gexec = nullptr;
    h->graph = nullptr;
  }
  return 0;
}

int mtsac_memcpy(void* dst, const void* src, int64_t bytes) {
  if (!dst || !src || bytes < 0) return fail(-22, "bad copy arguments");
  HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
  // a pageable-host -> device copy may still be in flight when hipMemcpy returns; the engine's
  // streams are non-blocking, so finish it before a hook hands the buffer back
  HIP_TRY(hipStreamSynchronize(nullptr));
  return 0;
}

// ---------------------------------------------------------------- timing
int mtsac_set_timing(mtsac_engine* h, int32_t enable) {
  if (!h) return fail(-22, "null engine");
  h->timing = enable != 0;
  h->timing_serial = enable == 2;
  return 0;
}
int mtsac_get_timing(mtsac_engine* h, int32_t family, double* total_ms, int32_t* launches, double* flops) {
  if (!h || !total_ms || !launches || !flops) return fail(-22, "null argument");
  HIP_TRY(hipStreamSynchronize(h->st));
  double ms = 0.0, fl = 0.0;
  int nl = 0;
  for (size_t i = 0; i < h->tl_next && i < h->tl.size(); ++i) {
    if (h->tl[i].family != family) continue;
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, h->tl[i].a, h->tl[i].b));
    ms += t;
    fl += h->tl[i].flops;
    ++nl;
  }
  *total_ms = ms;
  *launches = nl;
  *flops = fl;
  return 0;
}

int mtsac_get_timing_kernel(mtsac_engine* h, int32_t family, char* buf, int32_t n) {
  if (!h || !buf || n < 1) return fail(-22, "null argument");
  if (family < 0 || family >= 8) return fail(-22, "unknown family");
  std::snprintf(buf, (size_t)n, "%s", h->fam_kernel[family].c_str());
  return 0;
}

// ---------------------------------------------------------------- debug (include/mtsac_debug.h)
int mtsac_debug_set_pipeline(mtsac_engine* h, int32_t on) {
  if (!h) return fail(-22, "null engine");
  const int was = h->pipeline_req;
  h->pipeline_req = on < 0 ? -1 : on != 0 ? 1 : 0;
  return was;
}

int mtsac_debug_set_collective_model(mtsac_engine* h, int32_t nranks, double bus_gbps, int32_t flags) {
  if (!h) return fail(-22, "null engine");
  if (h->comm || h->hook || h->chook) return fail(-16, "a communicator or collective hook is installed");
  if (nranks < 1 || (nranks > 1 && !(bus_gbps > 0.0))) return fail(-22, "nranks >= 1 and bus_gbps > 0");
  HIP_TRY(hipStreamSynchronize(h->st));
  h->cmodel.nranks = nranks;
  h->cmodel.gbps = bus_gbps;
  h->cmodel.poison = (flags & 1) != 0;
  h->cmodel.blocks = ((flags >> 8) & 255) ? (flags >> 8) & 255 : 8;
  if (h->cmodel.poison) {  // the shadow holds the largest bucket: a whole trunk + the scalar tail
    long long need = 0;
    for (const Net* net : {&h->actor, &h->critic}) need = std::max(need, net->n_flat - net->trunk_off + EXTRA);
    if (need > h->cm_cap) {
      int rc = h->alloc(&h->cm_shadow, (size_t)need);
      if (rc) return rc;
      h->cm_cap = need;
    }
  }
  if (h->gexec) {  // the step's structure changed (buckets, sharded reductions)
    (void)hipGraphExecDestroy(h->gexec);
    (void)hipGraphDestroy(h->graph);
    h->gexec = nullptr;
    h->graph = nullptr;
  }
  return 0;
}

int mtsac_debug_force_one_stream(mtsac_engine* h, int32_t on) {
  if (!h) return fail(-22, "null engine");
  HIP_TRY(hipStreamSynchronize(h->st));
  mtsac_engine::Registry& r = mtsac_engine::registry();
  std::lock_guard<std::mutex> g(r.mu);
  h->force_one = on != 0;
  mtsac_engine::relane(r);
  return 0;
}

int mtsac_debug_set_bfrag(int32_t mode) {
  if (mode < -1 || mode > 1) return fail(-22, "bfrag mode is -1, 0 or 1");
  g_bfrag_mode = mode;
  return 0;
}

int mtsac_debug_bfrag(mtsac_engine* h) {
  if (!h) return fail(-22, "null engine");
  int m = 0;
  for (int i = 0; i < MAXD && i < 8; ++i) m |= (h->actor.bfrag[i] ? 1 << i : 0) | (h->critic.bfrag[i] ? 256 << i : 0);
  return m;
}

// MTSAC_GUARD_BYTES debug mode: the allocations whose guard zones a kernel wrote; returns their count
// (0: every guard intact, -95 when the mode is off) and names the first few (source line of the
// alloc call, side, first written byte) in mtsac_last_error
int mtsac_debug_check_guards(mtsac_engine* h) {
  if (!h) return fail(-22, "null engine");
  const size_t G = mtsac_engine::guard_bytes();
  if (G == 0) return fail(-95, "guard zones are off (set MTSAC_GUARD_BYTES before the engine is created)");
  HIP_TRY(hipDeviceSynchronize());
  std::vector<unsigned char> buf(G);
  int bad = 0;
  std::string msg;
  for (const auto& g : h->guards)
    for (int side = 0; side < 2; ++side) {
      HIP_TRY(hipMemcpy(buf.data(), g.base + (side ? G + g.bytes : 0), G, hipMemcpyDeviceToHost));
      size_t first = G, n = 0;
      for (size_t i = 0; i < G; ++i)
        if (buf[i] != 0xFF) {
          if (first == G) first = i;
          ++n;
        }
      if (n) {
        ++bad;
        if (bad <= 8)
          msg += "alloc@line " + std::to_string(g.line) + " (" + std::to_string(g.bytes) + " B) " +
                 (side ? "back" : "front") + " guard: " + std::to_string(n) + " bytes written, first at " +
                 (side ? "+" : "-") + std::to_string(side ? first : G - first) + "; ";
      }
    }
  if (bad) g_last_error = msg;
  return bad;
}

// Debug views of step buffers (tools/shard_diag.py).  mtsac_debug_snapshot(on): from the next step on,
// copy the actor's top activations right after the actor forward and after the actor-loss pass.
// mtsac_debug_read(id): 0 the actor's top activations now, 1 / 2 the two snapshots ([Ma][W] each),
// 3 the actor head's output gradient dout ([B][2A]), 4 the actor gradient's head leaves.
int mtsac_debug_snapshot(mtsac_engine* h, int32_t on) {
  if (!h) return fail(-22, "null engine");
  if (on && !h->dbg_snap[0])  // allocated once, reused when snapshots are turned on again (freed with the engine)
    for (float*& q : h->dbg_snap)
      if (int rc = h->alloc(&q, (size_t)h->Ma * h->actor.width)) return rc;
  h->snap_on = on != 0;
  return 0;
}

// The head backward's LDS self-check, tested: re-run the actor head's weight pass of the last step on
// its own buffers with one cross-wave LDS slot corrupted on purpose, into a scratch output (the
// gradients are untouched); the engine's next check_err (mtsac_get_logs / mtsac_synchronize) must then
// report HEAD_FAULT_WGRAD.  Needs a step first (the row lists and dout of the last step).
int mtsac_debug_head_selfcheck(mtsac_engine* h) {
  if (!h) return fail(-22, "null engine");
  if (h->actor.hd != 8 || h->actor.width % 4 != 0 || h->counts == nullptr) return fail(-95, "needs hd 8, W % 4 == 0 and a step");
  if (!h->dbg_hw)
    if (int rc = h->alloc(&h->dbg_hw, (size_t)h->T_l * h->actor.width * 8 + (size_t)h->T_l * 8)) return rc;
  const HeadParams ahp = h->head(h->actor, h->actor.p, h->ha[h->actor.depth - 1], h->B, h->task);
  head_backward_weight_inject(ahp, h->dout_a, 0, h->counts, h->rows, h->B, h->T_l, h->dbg_hw,
                              h->dbg_hw + (size_t)h->T_l * h->actor.width * 8, h->st);
  HIP_TRY(hipGetLastError());
  return 0;
}

int mtsac_debug_read(mtsac_engine* h, int32_t id, float* dst, int64_t count) {
  if (!h || !dst) return fail(-22, "null argument");
  const float* src = nullptr;
  int64_t n = 0;
  switch (id) {
    case 0: src = h->ha[h->actor.depth - 1]; n = (int64_t)h->Ma * h->actor.width; break;
    case 1: src = h->dbg_snap[0]; n = (int64_t)h->Ma * h->actor.width; break;
    case 2: src = h->dbg_snap[1]; n = (int64_t)h->Ma * h->actor.width; break;
    case 3: src = h->dout_a; n = (int64_t)h->B * 2 * h->A; break;
    case 4: src = h->actor.g; n = h->actor.trunk_off; break;
    default: return fail(-22, "unknown buffer id");
  }
  if (!src) return fail(-22, "buffer not allocated (mtsac_debug_snapshot)");
  if (count != n) return fail(-22, "count must be " + std::to_string(n));
  HIP_TRY(hipStreamSynchronize(h->st));
  HIP_TRY(hipMemcpy(dst, src, sizeof(float) * n, hipMemcpyDeviceToHost));
  return 0;
}

int mtsac_debug_lane_mode(mtsac_engine* h) {
  if (!h) return fail(-22, "null engine");
  return h->one_stream ? 1 : 0;
}

int mtsac_debug_timed_launch(mtsac_engine* h, int32_t i, int32_t* dims, double* ms) {
  if (!h) return fail(-22, "null engine");
  if (i < 0) return (int)std::min(h->tl_next, h->tl.size());
  if ((size_t)i >= std::min(h->tl_next, h->tl.size()) || !dims || !ms) return fail(-22, "bad launch index");
  HIP_TRY(hipStreamSynchronize(h->st));
  const auto& t = h->tl[i];
  dims[0] = t.family;
  dims[1] = t.M;
  dims[2] = t.N;
  dims[3] = t.K;
  dims[4] = t.batch;
  float v = 0.f;
  HIP_TRY(hipEventElapsedTime(&v, t.a, t.b));
  *ms = v;
  return 0;
}

int mtsac_debug_gemm(int precision, int kind, int epi, int batch, int M, int N, int K, const float* A, int lda, int a_shared,
                     const float* B, int ldb, float* C, int ldc, const float* bias, const float* mask, int ldm,
                     float* db) {
  const int splits = (precision >> 8) & 255;
  precision &= 255;
  if (kind < 0 || kind > 2 || batch < 1 || M < 1 || N < 1 || K < 1) return fail(-22, "bad gemm arguments");
  const bool ta = kind == 2, tb = kind == 1;
  const long long a_rows = ta ? K : M, b_rows = tb ? N : K;
  const long long sA = a_rows * lda, sB = b_rows * ldb, sC = (long long)M * ldc;
  float *dA = nullptr, *dB = nullptr, *dC = nullptr, *dbias = nullptr, *dmask = nullptr, *ddb = nullptr, *dws = nullptr;
  auto cleanup = [&]() {
    for (float* p : {dA, dB, dC, dbias, dmask, ddb, dws})
      if (p) (void)hipFree(p);
  };
  const long long nA = a_shared ? sA : sA * batch;
  bool ok = hipMalloc(&dA, sizeof(float) * nA) == hipSuccess && hipMalloc(&dB, sizeof(float) * sB * batch) == hipSuccess &&
            hipMalloc(&dC, sizeof(float) * sC * batch) == hipSuccess;
  if (ok && bias) ok = hipMalloc(&dbias, sizeof(float) * N * batch) == hipSuccess;
  if (ok && mask) ok = hipMalloc(&dmask, sizeof(float) * (long long)M * ldm * batch) == hipSuccess;
  if (ok && db) ok = hipMalloc(&ddb, sizeof(float) * N * batch) == hipSuccess;
  if (ok && splits > 1) ok = hipMalloc(&dws, sizeof(float) * gemm_ws_floats(M, N, batch, splits)) == hipSuccess;
  if (!ok) {
    cleanup();
    return fail(-12, "hipMalloc failed");
  }
  (void)hipMemcpy(dA, A, sizeof(float) * nA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, sizeof(float) * sB * batch, hipMemcpyHostToDevice);
  (void)hipMemcpy(dC, C, sizeof(float) * sC * batch, hipMemcpyHostToDevice);
  if (bias) (void)hipMemcpy(dbias, bias, sizeof(float) * N * batch, hipMemcpyHostToDevice);
  if (mask) (void)hipMemcpy(dmask, mask, sizeof(float) * (long long)M * ldm * batch, hipMemcpyHostToDevice);
  GemmParams g{};
  g.A = dA; g.lda = lda; g.sA = a_shared ? 0 : sA;
  g.B = dB; g.ldb = ldb; g.sB = sB;
  g.C = dC; g.ldc = ldc; g.sC = sC;
  g.bias = dbias; g.sBias = N;
  g.mask = dmask; g.ldm = ldm; g.sMask = (long long)M * ldm;
  g.db = ddb; g.sDb = N;
  g.M = M; g.N = N; g.K = K;
  g.splits = splits;
  g.ws = dws;
  if (precision == MTSAC_FP32_SPLIT3)
    gemm_x3(g, (GemmKind)kind, epi, batch, nullptr);
  else
    gemm_f32(g, (GemmKind)kind, epi, batch, nullptr);
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(C, dC, sizeof(float) * sC * batch, hipMemcpyDeviceToHost);
  if (e == hipSuccess && db) e = hipMemcpy(db, ddb, sizeof(float) * N * batch, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) return fail(-5, std::string("debug gemm: ") + hipGetErrorString(e));
  return 0;
}

__global__ void fill_rand_kernel(float* p, long long n, unsigned seed) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = ((float)(x & 0xFFFFFF) / 8388608.0f) - 1.0f;
}

int mtsac_debug_gemm_bench(int precision, int kind, int epi, int batch, int M, int N, int K, int iters,
                           double* ms_per_launch) {
  const int splits = (precision >> 8) & 255;
  precision &= 255;
  if (kind < 0 || kind > 2 || batch < 1 || M < 1 || N < 1 || K < 1 || iters < 1 || !ms_per_launch)
    return fail(-22, "bad gemm bench arguments");
  const bool ta = kind == 2, tb = kind == 1;
  const int lda = ta ? M : K, ldb = tb ? K : N;
  const long long sA = (long long)(ta ? K : M) * lda, sB = (long long)(tb ? N : K) * ldb, sC = (long long)M * N;
  float *A = nullptr, *B = nullptr, *C = nullptr, *bias = nullptr, *db = nullptr, *ws = nullptr;
  if (splits > 1) HIP_TRY(hipMalloc(&ws, sizeof(float) * gemm_ws_floats(M, N, batch, splits)));
  HIP_TRY(hipMalloc(&A, sizeof(float) * sA * batch));
  HIP_TRY(hipMalloc(&B, sizeof(float) * sB * batch));
  HIP_TRY(hipMalloc(&C, sizeof(float) * sC * batch));
  HIP_TRY(hipMalloc(&bias, sizeof(float) * N * batch));
  HIP_TRY(hipMalloc(&db, sizeof(float) * N * batch));
  for (auto pr : {std::make_pair(A, sA * batch), std::make_pair(B, sB * batch), std::make_pair(C, sC * batch),
                  std::make_pair(bias, (long long)N * batch)})
    hipLaunchKernelGGL(fill_rand_kernel, dim3((unsigned)((pr.second + 255) / 256)), dim3(256), 0, nullptr,
                       pr.first, pr.second, 17u);
  GemmParams g{};
  g.A = A; g.lda = lda; g.sA = sA;
  g.B = B; g.ldb = ldb; g.sB = sB;
  g.C = C; g.ldc = N; g.sC = sC;
  g.bias = bias; g.sBias = N;
  g.mask = C; g.ldm = N; g.sMask = sC;  // any sign pattern will do
  g.db = (kind == 2) ? db : nullptr; g.sDb = N;
  g.M = M; g.N = N; g.K = K;
  g.splits = splits;
  g.ws = ws;
  auto launch = [&]() {
    if (precision == MTSAC_FP32_SPLIT3)
      gemm_x3(g, (GemmKind)kind, epi, batch, nullptr);
    else
      gemm_f32(g, (GemmKind)kind, epi, batch, nullptr);
  };
  launch();
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i) launch();
  HIP_TRY(hipEventRecord(e1, nullptr));
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  *ms_per_launch = ms / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  for (float* p : {A, B, C, bias, db, ws})
    if (p) (void)hipFree(p);
  return 0;
}

}  // extern "C"
