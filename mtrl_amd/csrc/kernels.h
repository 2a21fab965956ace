// kernels.h -- launch wrappers of the MTSAC device kernels (internal to libmtsac.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtsac {

// ------------------------------------------------------------------ GEMM
// C[z] = op(A[z]) . op(B[z]) with a fused epilogue, fp32 in / fp32 accumulate on
// v_mfma_f32_32x32x2_f32.  TA: A stored [K][M] (else [M][K]); TB: B stored [N][K]
// (else [K][N]).  Leading dims and base pointers must be multiples of 4 floats.
enum GemmEpi {
  EPI_STORE = 0,      // C = acc                       (weight grads; + optional db column sums)
  EPI_BIAS_RELU = 1,  // C = max(acc + bias[n], 0)     (trunk forward)
  EPI_RELU_MASK = 2,  // C = acc * (mask[m][n] > 0)    (data grad through the previous ReLU)
};

struct GemmParams {
  const float* A;
  const float* B;
  float* C;
  const float* bias;  // EPI_BIAS_RELU
  const float* mask;  // EPI_RELU_MASK
  float* db;          // EPI_STORE + TB==false: column sums of B (bias gradient), may be null
  int M, N, K;
  int lda, ldb, ldc, ldm;
  long long sA, sB, sC, sBias, sMask, sDb;  // per-batch strides (elements)
  // split-K (EPI_STORE only): `splits` slices of K write dense partials (and db partials) into
  // ws, then a fixed-order reduction writes C / db.  ws needs gemm_ws_floats() floats.
  int splits;
  int kchunk;                               // set by the launcher
  float* ws;
  // gemm_x3 only: also write the bf16 split planes of C ([3][M][ldcp] per batch entry)
  __bf16* Cp;
  long long ldcp, pC, sCp;
};

enum GemmKind { GEMM_NN = 0, GEMM_NT = 1, GEMM_TN = 2 };
// K slices that fill the chip for an EPI_STORE GEMM with few output tiles (1 = no split)
int gemm_splits(int M, int N, int K, int batch);
long long gemm_ws_floats(int M, int N, int batch, int splits);
// C[z] = sum_s ws[z*S + s] (+ db likewise), fixed order: deterministic
// everything after a split-K GEMM in one launch: the slab sums into C, the per-slice bias sums
// (p.db), and optionally a bias grad finished from column-sum partials cs_part [batch][chunks][N]
struct ReduceJob {
  const float* ws;
  int S, M, N;
  float* C;
  int ldc;
  long long sC;
  const float* dbws;
  float* db;
  long long sDb;
  const float* cs_part;
  int cs_chunks;
  float* cs_db;
  long long cs_sdb;
};
void splitk_reduce(const GemmParams& p, int batch, int splits, hipStream_t st, const float* cs_part = nullptr,
                   int cs_chunks = 0, float* cs_db = nullptr, long long cs_sdb = 0);
// A weight grad's finish (split-K slab sums and / or the bias grad from column-sum partials), collected
// instead of launched (SplitGemmParams::defer) and run with the network's other ones in ONE launch
// before its optimizer (finish_many): the same blocks, sums and order as splitk_finish_all_kernel.
struct DeferredFinish {
  ReduceJob j;
  int nred, ndb, ncs;
};
constexpr int FINISH_SINK_JOBS = 8;
struct FinishSink {
  DeferredFinish job[FINISH_SINK_JOBS];
  int n = 0;
};
// the job splitk_reduce launches (nred + ndb + ncs blocks per batch entry)
DeferredFinish reduce_job(const GemmParams& p, int batch, int splits, const float* cs_part, int cs_chunks,
                          float* cs_db, long long cs_sdb);
// a bias grad from column-sum partials only (what colsum_finish launches)
DeferredFinish colsum_job(const float* part, int cols, int chunks, float* db, long long sdb);
// every job of the sink in one launch (batch entries: grid.y), then the sink is empty
void finish_many(FinishSink& s, int batch, hipStream_t st);
// out[z][c][r] = in[z][r][c]  (rows x cols per batch entry, dense)
void transpose_f32(const float* in, long long s_in, float* out, long long s_out, int rows, int cols, int batch,
                   hipStream_t st);
void gemm_f32(const GemmParams& p, GemmKind kind, int epi, int batch, hipStream_t st);
// same contract, fp32-accurate via 3-way bf16 operand split on bf16 MFMA (gemm_x3.hip)
void gemm_x3(const GemmParams& p, GemmKind kind, int epi, int batch, hipStream_t st);

// ------------------------------------------------------------------ split2h plane records
// Device record of one fp16-plane tensor (precision split2h): the planes hold x * 2^e; amax holds
// the partial maxima |x| of the last write, one per producer workgroup (the host knows how many are
// valid).  Weight records keep amax[0] = max |trunk parameter| (kernels and biases), amax[1] = max
// |head parameter| (the optimizer's last workgroup reduces them).
constexpr int PLANE_REC_PARTS = 2048;
struct PlaneRec {
  int e;
  int pad[3];
  float amax[PLANE_REC_PARTS];
};

// ------------------------------------------------------------------ pre-split plane GEMM
// C[z][m][n] = sum_k A(m,k) B(n,k) on bf16 planes (gemm_x3p.hip).  A planes [3][M][lda]
// (k contiguous) or, with a_kmajor, [3][K][lda] (m contiguous); B likewise with N.  K is a
// multiple of 32 (row-major planes zero-padded to it); lda/ldb multiples of 8.
struct SplitGemmParams {
  const __bf16* A;
  long long lda, pA, sA;  // row stride, plane stride, batch stride (elements)
  const __bf16* B;
  long long ldb, pB, sB;
  int a_kmajor, b_kmajor;
  float* C;               // fp32 output (may be null when only planes are wanted)
  int ldc;
  long long sC;
  const float* bias;
  long long sBias;
  const float* mask;
  int ldm;
  long long sMask;
  const __bf16* mask16;   // gemm_x3f: ReLU mask from the bf16 high plane [rows][ldm] instead of mask
  __bf16* Cp;             // optional split planes of C: [3][M][ldcp]
  long long ldcp, pC, sCp;
  int M, N, K;
  int splits, kchunk;     // split-K: partial slabs in ws (gemm_x3p_ws_floats), then a finishing pass; -1 = auto
  float* ws;
  int dbg;                // experiments only: bit0 skip steady-state loads, bit1 skip MFMA
  int tag;                // 1: input-layer launch (separate kernel symbol for profiles)
  int order;              // gemm_x3f tile order inside an XCD's run: 0 column tiles fastest, 1 row tiles
                          // fastest (experiments: MTSAC_X3F_ORDER)
  int b_frag;             // gemm_x3f: B planes in the fragment layout (frag_off: every 16-row x 32-k
                          // MFMA fragment 1 KB contiguous, so a B wave load reads 8 whole lines)
  int np;                 // operand planes the products read: 3 (0 = default; fp32-accurate split) or 1
                          // (precision bf16: the high plane only, one MFMA per product)
  float* dbp;             // gemm_x3f: column sums of the epilogue's output per row tile, [z][row tiles][N]
                          // (the next weight grad's bias grad, finished by colsum_finish), or null
  const float* cs_part;   // gemm_x3p EPI_STORE: also finish a bias grad from column-sum partials
  int cs_chunks;          // [batch][cs_chunks][N] (folded into the split-K reduce launch), or null
  float* cs_db;
  long long cs_sdb;
  int* cnt;               // gemm_x3f split-K: per-tile arrival counters (zero, >= GEMM_X3F_CNT ints) for
                          // the in-launch finish, or null (a separate finishing pass)
  // ---- precision split2h (np == 2): every operand is two fp16 planes of x * 2^e with e per tensor
  // (PlaneRec); the products are unscaled by 2^-(eA + eB).  Output planes are written at the exponent
  // of the a-priori bound  kmul * max|A| * max|B| (+ max|B| again when the bias lives in B's record:
  // the trunk's biases are bounded by the same trunk maximum), which every workgroup derives alike
  // from the operands' records; workgroup 0 stores it in rc->e and every workgroup its max |out| in
  // rc->amax[blockIdx.x] (the next producer's bound input).
  const PlaneRec* ra;
  int na;                 // valid partial maxima in ra (0: the bound 2^(15 - e) of its planes)
  const PlaneRec* rb;
  int nb;
  PlaneRec* rc;
  int bias_in_b;
  float kmul;             // the number of terms in each output sum (unpadded K)
  long long pMask;        // plane stride of the mask16 planes (np == 2: x > 0 <=> hi > 0 or lo > 0)
  int* nparts;            // host: the launcher stores how many partial maxima it wrote to rc (or null)
  FinishSink* defer;      // host, gemm_x3p EPI_STORE: collect the finish (slab sums, bias grad) here
                          // instead of launching it (null: launch), when the sink has room
};
constexpr int GEMM_X3F_CNT = 4096;
void gemm_x3p(const SplitGemmParams& p, int epi, int batch, hipStream_t st);
// split-K finishing pass: C / Cp = epi(sum over the S slabs of p.ws, in slice order); the ReLU mask
// from p.mask16 when set, else p.mask
void splitk_finish(const SplitGemmParams& p, int epi, int S, int batch, hipStream_t st);
// auto split-K slices (1 = none) for a plane GEMM; kmajor = the k-major x k-major form
// np: operand planes (1 = bf16 picks its own weight-grad tiles); the default sizes for the widest form
int gemm_x3p_splits(int M, int N, int K, int batch, bool kmajor, int np = 3);
long long gemm_x3p_ws_floats(int M, int N, int K, int batch, bool kmajor);
// row-major x row-major plane GEMM on 16x16x32 MFMA, 208 x 256 tiles (gemm_x3f.hip): forward
// (EPI_BIAS_RELU) and data grad (EPI_RELU_MASK) when gemm_x3f_ok
bool gemm_x3f_ok(const SplitGemmParams& p, int epi, int batch);
int gemm_x3f(const SplitGemmParams& p, int epi, int batch, hipStream_t st);  // returns the K slices used
int gemm_x3f_tiles(int M, int N, int batch);
int gemm_x3f_row_tiles(int M);  // row tiles of M (the dbp partials' chunk count)
int gemm_x3f_bm(const SplitGemmParams& p, int batch);  // row tile of an unsplit launch (208; bf16: 48..400)
int gemm_x3f_max_row_tiles(int M);  // row tiles of M at the shortest tile (dbp partial buffers)
// split-K for few rows: slices (1 = none) and workspace floats; gemm_x3f splits when the params
// allow it (splits < 0, ws given, no dbp)
int gemm_x3f_splits(int M, int N, int K, int batch);
int gemm_x3f_split_bm(int M, int N, int K, int batch);  // row tile of the split-K launches (208 or 128)
int gemm_x3f_out_bm(const SplitGemmParams& p, int epi, int batch);  // row tile of the launch gemm_x3f makes
long long gemm_x3f_ws_floats(int M, int N, int K, int batch);
void gemm_x3f_ablate(const SplitGemmParams& p, int abl, int batch, hipStream_t st);  // experiments
// the same contract for small row counts (task shards, MT10): 16 TI x 64 tiles, 4 waves splitting
// K inside the workgroup (gemm_x3s.hip); the ReLU mask comes from mask16
bool gemm_x3s_ok(const SplitGemmParams& p, int epi, int batch);
void gemm_x3s(const SplitGemmParams& p, int epi, int batch, hipStream_t st);
int gemm_x3s_ti(int M, int N, int batch);
void gemm_x3s_ablate(const SplitGemmParams& p, int abl, int batch, hipStream_t st);  // experiments
extern int g_x3p_geo;  // tile geometry of gemm_x3p (-1: by operand form, 0..3: forced; see gemm_x3p.hip)
extern int g_x3p_dbg;  // experiment bits OR-ed into SplitGemmParams::dbg
extern int g_x3_dbg;   // experiments on gemm_x3: bit0 skip loads after the first tile, bit1 skip MFMA, bit2 skip split

// fp32 x[z][rows][ldx] -> bf16 planes out[z][3][out_rows][ldo] (plane stride po); TRANSPOSE
// writes out[q][col][row].  Elements past rows/cols inside [out_rows, out_cols) become 0.
struct SplitParams {
  const float* x;
  long long ldx, sx;
  int rows, cols;
  __bf16* out;
  long long ldo, po, so;
  int out_rows, out_cols;
  const int* e2h;  // non-null: precision split2h, two fp16 planes of x * 2^(*e2h) (gemm_common.h split2h_dev)
  int frag;        // out planes in the fragment layout (gemm_common.h frag_off; ldo % 32 == 0, out_rows % 16 == 0)
};
void split_planes(const SplitParams& s, bool transpose, int batch, hipStream_t st);
// db[z][c] = sum_r x[z][r][c] (deterministic two-pass; part holds batch*COLSUM_CHUNKS*cols floats)
constexpr int COLSUM_CHUNKS = 64;
// db[z][c] = sum over chunks (in order) of part[z][chunks][cols]: the second pass of colsum for
// partials written by a producing kernel's epilogue (head backward, gemm_x3f data grad)
void colsum_finish(const float* part, int cols, int chunks, int batch, float* db, long long sdb, hipStream_t st);
void colsum(const float* x, int rows, int cols, int ld, long long sx, int batch, float* part, float* db,
            long long sdb, hipStream_t st);

// ------------------------------------------------------------------ replay
struct PcgDev {  // device-resident numpy PCG64 state (buffers.py:260)
  unsigned long long state_hi, state_lo, inc_hi, inc_lo;
  int has_uint32;
  unsigned int uinteger;
};
// n indices in [0, max(size, n)) with numpy's Generator.integers stream; size read from *buf_size
void replay_indices(PcgDev* rng, const unsigned long long* jump /*65 x (A_hi,A_lo,C_hi,C_lo)*/,
                    const long long* buf_size, int n, int* idx_out, hipStream_t st);
// the same stream for integers(0, high) with high given (>= 1; high == 1 draws nothing)
void replay_indices_high(PcgDev* rng, const unsigned long long* jump, long long high, int n, int* idx_out,
                         hipStream_t st);

struct GatherParams {
  const float* store;   // [cap][T_l][R] transition records
  const int* idx;       // [n]
  int n, T_l, R, obs_dim, act_dim, T_glob, task_begin;
  int ld_a, ld_c;       // padded widths of actor / critic inputs
  float* xa;            // [B][ld_a]  obs
  float* xa_next;       // [B][ld_a]  next_obs
  float* xc;            // [B][ld_c]  (action | obs)
  float* xc_next;       // [B][ld_c]  (a' | next_obs), a' columns written later
  float* xc_pi;         // [B][ld_c]  (a | obs), a columns written later
  float* rew;           // [B]
  float* done;          // [B]
  int* task;            // [B] local task id
  const double* rmin;   // per-task reward min/max (normalize_rewards) or null
  const double* rmax;
  double norm_eps;
  int* err;             // error flag (one-hot violation)
  // bf16 planes of the GEMM inputs (split3 / bf16 engines; null otherwise), written beside the fp32
  // rows so no split pass runs before the trunk forward: xa's [3][.][pa_ld] (s rows at b, s' rows at
  // pa_next + b), xc / xc_next / xc_pi's [3][.][pc_ld] (the a' / a columns come from the policy head)
  __bf16* pa;
  long long pa_ps, pa_next;
  int pa_ld;
  __bf16 *pc, *pcn, *pcp;
  long long pc_ps;
  int pc_ld;
  // split2h: fp16 planes at the exponent of max(*in_max, 1) (the stored rows' max |value|; 1 covers the
  // policy's actions), written to in_rec->e
  PlaneRec* in_rec;
  const float* in_max;
};
void replay_gather(const GatherParams& p, hipStream_t st);
// a user batch (ReplayBufferSamples layout) into the same input buffers
void batch_scatter(const GatherParams& p, const float* obs, const float* act, const float* nobs,
                   const float* done, const float* rew, int B, hipStream_t st);
// async add (engine.cpp mtsac_buffer_add): pack a slot from device arrays; commit it (reward
// min/max, sampled range) on the device
void buffer_pack_slot(float* rec, int T_l, int R, int D, int A, const float* obs, const float* nobs,
                      const float* act, const float* rew, const float* done, hipStream_t st);
void buffer_commit_slot(const float* rec, int T_l, int R, int rcol, double* rmin, double* rmax, long long* buf_size,
                        long long size, hipStream_t st, int D = 0, float* bufmax = nullptr);
// bufmax (nullable): *bufmax = max(*bufmax, max |obs|, |action|, |next_obs| written) -- split2h's input bound
void fill_synthetic(float* store, long long cap, int T_l, int R, int obs_dim, int act_dim, int T_glob,
                    int task_begin, unsigned long long seed, hipStream_t st, float* bufmax = nullptr);
// *m = max(*m, max |x[0..n)|) (one block)
void absmax_into(const float* x, long long n, float* m, hipStream_t st);
// stable per-task row lists: rows_of[t*max_rows + j], counts[t]
void task_rows(const int* task, int B, int T_l, int* counts, int* rows, int max_rows, hipStream_t st);

// ------------------------------------------------------------------ heads / policy / losses
struct HeadParams {
  const float* h;       // [E][B][W] last trunk activation
  const float* Wh;      // [E][T_l][W][hd]
  const float* WhT;     // [T_l][hd][W]: Wh transposed per task (the actor's, E = 1), or null: the policy
                        // heads' weight loads then read whole lines (Wh rows are hd floats apart)
  const float* bh;      // [E][T_l][hd]
  const int* task;      // [B]
  int B, W, hd, E;
  long long sWh, sbh, sh;
  unsigned* fault;      // nullable: the head backward's LDS-reduction self-checks OR a bit in here on a
                        // mismatch (HEAD_FAULT_*); the engine reports it at the next sync (check_err)
};
// HeadParams::fault bits: which checked cross-wave LDS reduction saw a slot differ from its writer's bits
constexpr unsigned HEAD_FAULT_WGRAD = 1u;   // the head weight grad's four-wave sum
constexpr unsigned HEAD_FAULT_COLSUM = 2u;  // the data pass's per-row-slice column sums (bias-grad partials)

// actor head + tanh-normal sample (networks.py:28-45, distributions.py:6-16)
struct PolicyParams {
  HeadParams head;
  const float* eps;     // [B][A] injected noise or null (device stream)
  unsigned long long seed;
  const unsigned long long* counter;  // device step counter (noise stream position)
  unsigned int stream_id;
  int A;
  float ls_min, ls_max;
  float* a_out;         // written at [b*ld_a_out + j]
  int ld_a_out;
  float* a_out2;        // optional second copy
  int ld_a_out2;
  __bf16* a_planes;     // optional bf16 planes of a_out's action columns ([3][.][ap_ld], plane stride ap_ps)
  long long ap_ps;
  int ap_ld;
  const PlaneRec* ap_rec;  // split2h: the planes are fp16 at the input record's exponent (|a| <= 1 fits)
  float* logpi;         // [B]
  float* cache;         // optional [B][5A]: mu, ls, x, a, eps
  // optional per-task row lists (task_rows): rows grouped by task share head-kernel reads
  const int* counts;
  const int* rows;
  int max_rows, T_l;    // row-list stride, local tasks
  int max_count;        // bound on counts[] (sizes the grid)
};
void policy_head(const PolicyParams& p, hipStream_t st);
// WhT[t][o][w] = Wh[t][w][o] for T_l tasks (E = 1): the policy heads' copy, after every write of Wh
void head_transpose(const float* Wh, int T_l, int W, int hd, float* WhT, hipStream_t st);
// the s and s' heads of the merged actor forward in one launch (grouped form; else two launches)
struct PolicyPair {
  PolicyParams p[2];
};
void policy_head_pair(const PolicyParams& a, const PolicyParams& b, hipStream_t st);

enum CriticHeadMode { CH_TARGET = 0, CH_CRITIC = 1, CH_ACTOR = 2 };
struct CriticHeadParams {
  HeadParams head;      // E = num_critics, hd = 1
  int mode;
  HeadParams thead;     // CH_CRITIC with fused_target: the target critic's head at (s', a') first,
  int fused_target;     // y = TD target (logpi = logpi(a'|s'), written to y_out), in the same launch
  const float* rew;
  const float* done;
  const float* logpi;   // target: logpi(a'|s'); actor: logpi(a|s)
  const float* log_alpha;  // [T_glob]
  const int* task;
  int task_begin;
  const float* y;       // critic mode input
  float* y_out;         // target mode output
  float* dq;            // [E][B] dL/dq (critic, actor modes)
  float* row_a;         // per-row reduction inputs [B]
  float* row_b;         // [B]
  const float* tw;      // per-row task weights or null
  float* alpha_w;       // CH_ACTOR: per-row dL/dlogpi = w * alpha / B
  float gamma;
  int clip;
  int use_task_weights;
  int T_glob;
  float inv_norm;       // 1/(E*B) critic, 1/B actor (global B)
  PlaneRec* dq_rec;     // split2h: per-workgroup max |dq| (the head backward's bound input), or null
  int* dq_parts;        // host: how many the launch wrote
};
void critic_head(const CriticHeadParams& p, hipStream_t st);

// optional bf16 split planes of an output: [E][3][rows][ld], plane stride ps, member stride sm.
// split2h (rc non-null): two fp16 planes at the exponent of the bound  kmul * max|dout| * (max|head
// weight| + w_add)  (dout's record rd with nd partial maxima; the weights' record rw keeps max|head|
// in amax[1], w_add covers the optimizer steps since), per-workgroup maxima to rc
struct PlaneOut {
  __bf16* p;
  long long ld, ps, sm;
  PlaneRec* rc;
  const PlaneRec* rd;
  int nd;
  const PlaneRec* rw;
  float w_add, kmul;
  int* nparts;          // host: how many partial maxima the launch wrote
};
// dz[e][b][w] = (sum_o dout[e][b][o] * Wh[e][t_b][w][o]) * (h[e][b][w] > 0)  (+ its planes), rows
// walked per task (counts / rows of task_rows); dz may be null (planes only).  dbp (nullable):
// column sums of dz per (task, row slice), [e][head_backward_chunks(T_l)][W], finished by
// colsum_finish.  W % 4 == 0.
void head_backward_data(const HeadParams& hp, const float* dout, long long s_dout, float* dz, const int* counts,
                        const int* rows, int max_rows, int T_l, hipStream_t st, PlaneOut po = PlaneOut{},
                        float* dbp = nullptr);
int head_backward_chunks(int T_l);
// head_backward_data + head_backward_weight of one head in one launch (false: W % 4 != 0, not launched)
bool head_backward_both(const HeadParams& hp, const float* dout, long long s_dout, float* dz, const int* counts,
                        const int* rows, int max_rows, int T_l, PlaneOut po, float* dbp, float* dWh, float* dbh,
                        hipStream_t st);
// dWh[e][t][w][o] = sum_{b in t} h[e][b][w] dout[e][b][o];  dbh[e][t][o] = sum dout
// head_backward_weight with one cross-wave LDS slot corrupted on purpose (hd = 8 only): the self-check's
// test -- the engine's next check_err must report HEAD_FAULT_WGRAD (mtsac_debug_head_selfcheck)
void head_backward_weight_inject(const HeadParams& hp, const float* dout, long long s_dout, const int* counts,
                                 const int* rows, int max_rows, int T_l, float* dWh, float* dbh, hipStream_t st);
void head_backward_weight(const HeadParams& hp, const float* dout, long long s_dout, const int* counts,
                          const int* rows, int max_rows, float* dWh, float* dbh, hipStream_t st);

// critic data grad into the action columns + tanh-normal backward -> actor head grad
struct ActionGradParams {
  const float* dz1;     // [E][B][Wc]  grad at critic layer-0 pre-activation
  const float* W0;      // [E][Ic][Wc] critic layer-0 kernel (rows 0..A-1 = action)
  long long s_dz, s_W0;
  int E, B, Wc, A;
  const float* cache;   // [B][5A] from policy_head
  const float* alpha_w; // [B] per-row dL/dlogpi (alpha * w / B)
  float ls_min, ls_max;
  float* dout;          // [B][2A]
  PlaneRec* dout_rec;   // split2h: per-workgroup max |dout| (the head backward's bound input), or null
  int* dout_parts;      // host: how many the launch wrote
};
void action_grad(const ActionGradParams& p, hipStream_t st);

// per-row alpha (and task weights) from log_alpha (mtsac.py:60-63,103-113)
void row_alpha(const int* task, int task_begin, const float* log_alpha, int T_glob, int B,
               int use_task_weights, float* alpha_row, float* tw_row, hipStream_t st);

// ------------------------------------------------------------------ reductions / optimizer
// out[i] = sum over rows of in_i (deterministic single-block tree)
void reduce_rows(const float* const* ins, int n_in, int B, float* out, hipStream_t st);

// modelled collective (coll_model.hip): 2 (N - 1) / N * bytes over bus_gbps, held by `blocks`
// workgroups on the stream; shadow non-null: the bucket is NaN until the delay is over
double coll_model_us(long long bytes, int nranks, double bus_gbps);
void coll_model_allreduce(float* buf, long long count, int nranks, double bus_gbps, int blocks, float* shadow,
                          hipStream_t st, double scale = 1.0);
// partial sums of squares of x[0..n) into partials[grid]; returns grid size used
int sumsq_partials(const float* x, long long n, float* partials, int max_blocks, hipStream_t st);
// optimizer scalars: sums partials, computes norm and clip scale
struct OptScalars {
  float gnorm;          // pre-clip global norm
  float scale;          // clip factor applied to the gradient
  float pnorm;          // post-update parameter norm
  int count;            // adam step count (after increment)
};
void grad_norm_finalize(const float* partials, int nparts, const float* extra_sq /*nullable*/,
                        float max_norm, OptScalars* sc, hipStream_t st);
// bf16 split planes of updated parameters: flat p[begin, begin + members * member_n) is written
// as planes[e][q][k] (plane stride ps, member stride 3 * ps), k < member_n -- the natural-layout
// planes of a dense kernel leaf whose row stride equals its width
struct PlaneSeg {
  long long begin, member_n, members;
  __bf16* planes;
  long long ps;
  int of_target;        // 1: planes of the Polyak target's new value instead of the params'
};
// split2h (np == 2) weights: the optimizer writes fp16 planes of p * 2^e with e from the bound
// max|p_old| + w_add (w_add covers one Adam step, engine.cpp adam_step_bound: |m_hat| / sqrt(v_hat)
// <= 7.27 at b1 = 0.9, b2 = 0.999), the target's at max(max|t_old|, that), stores both exponents in the records and
// leaves per-block max |p_new| / |t_new| partials for step_finish to reduce into the records
struct WeightH2 {
  PlaneRec* wrec;       // params: e, amax[0] trunk max, amax[1] head max
  PlaneRec* trec;       // Polyak target (null: none)
  float w_add;
  float* wparts;        // per-block max |p_new| [grid]
  float* tparts;        // per-block max |t_new| [grid] (target)
};
constexpr int MAX_PLANE_SEGS = 8;
struct AdamParams {
  float* p; float* m; float* v; const float* g;
  float* target;        // polyak target (critic) or null
  long long n;
  float lr, b1, b2, eps, tau;
  OptScalars* sc;
  float* p_partials;    // sum of squares of new params per block
  int nseg;             // planes of the new params to write (offsets relative to p)
  PlaneSeg seg[MAX_PLANE_SEGS];
  int np;               // planes the GEMMs read: 1 (precision bf16) writes only the high plane
  int nskip;            // float4 ranges [skip_b, skip_e) of p left to adam_update_tiles
  long long skip_b[MAX_PLANE_SEGS], skip_e[MAX_PLANE_SEGS];
  WeightH2 h2;          // np == 2
  int refresh;          // 1: no Adam step -- p is already the new value (the sharded optimizer's all-gathered
                        // trunk); Polyak (target non-null), planes, |p|^2 and maxima as usual
  float* whT;           // the actor's head kernel transposed per task ([T][hd][W], heads.hip WhT) written
  long long whT_b4, whT_e4;  // from the new values of the float4 range [whT_b4, whT_e4) of p ([T][W][hd]),
  int whT_W, whT_hd;         // or null (then head_transpose rewrites it)
};
// p_partials accumulate |p_new|^2 over [norm_from, n) only (the replicated trunk range)
int adam_update(const AdamParams& a, float max_norm, long long norm_from, int max_blocks, hipStream_t st);
// The same update over dense kernel leaves [members][rows][cols] (cols % 4 == 0) in 64 x 64 tiles
// through LDS, writing the bf16 planes of the new params / target in the natural layout
// ([e][3][rows][nat_ld], the data grad's B) and transposed ([e][3][cols][tr_ld], k = row
// contiguous: the row-major forward's B) -- replaces the separate transposing split of
// refresh_wt.  Per-element arithmetic is adam_kernel's; |p_new|^2 partials, one per block, go to
// a.p_partials (blocks <= max_blocks).  Offsets relative to a.p.
struct TileLeaf {
  long long off, ms;    // first member's offset, member stride (floats)
  int rows, cols, members;
  int tiles_r, tiles_c, tile_begin;
  __bf16* nat[2];       // [0] params, [1] target (null: not wanted)
  long long nat_ld, nat_ps;
  __bf16* tr[2];
  long long tr_ld, tr_ps;
  int frag;  // nat and tr planes in the fragment layout (gemm_common.h frag_off)
};
constexpr int MAX_TILE_LEAVES = 8;
struct TileParams {
  int n, total;
  TileLeaf leaf[MAX_TILE_LEAVES];
};
int adam_update_tiles(const AdamParams& a, const TileParams& tp, float max_norm, int max_blocks, hipStream_t st);
// s0->pnorm = sqrt(trunk_sq[0] + head_sq[0]); s1 likewise with index 1
void pnorm_finalize(const float* trunk_sq, const float* head_sq, OptScalars* s0, OptScalars* s1, hipStream_t st);
// *out = sum(partials)  (one block, double accumulation)
void sum_partials(const float* partials, int nparts, float* out, hipStream_t st);
void adam_count_incr(OptScalars* sc, hipStream_t st);
// Fused optimizer step of one network (two launches): sumsq2 writes the |g|^2 partials of the heads'
// range [hparts, gh of them; h null: none] and the trunk's [tparts, returned count] and bumps the
// Adam count; adam_fused recomputes the global norm in every block (trunk partials + head partials,
// or the all-reduced head |g|^2 when head_sq is set), then updates the heads (ah) elementwise and
// the trunk (at) elementwise + in 64 x 64 tiles (tp; total 0: none), |p_new|^2 partials to ph / pt.
constexpr int FUSED_HEAD_PARTS = 256;
struct FusedOpt {
  const float* gparts; int ng;      // trunk |g|^2 partials
  const float* hparts; int nh;      // head |g|^2 partials (unsharded) ...
  const float* head_sq;             // ... or the all-reduced head |g|^2 (sharded), else null
  float max_norm;
  float *ph, *pt;                   // |p_new|^2 partials out: heads [bh], trunk [bt + btile]
  int bh, bt, btile;                // set by adam_fused
};
int sumsq2(const float* h, long long nh, const float* t, long long nt, float* hparts, float* tparts, OptScalars* sc,
           int* gh_out, hipStream_t st);
void adam_fused(const AdamParams& ah, const AdamParams& at, const TileParams& tp, FusedOpt& f, hipStream_t st);
// Sharded trunk optimizer (ZeRO-1, engine.cpp optimize_zero): |g|^2 over this rank's shard of every
// reduce-scattered bucket, added to *out (partials summed in a fixed order), and the Adam count bumped
struct ShardRanges {
  long long b[8], e[8];  // float4 index ranges of g
  int n;
};
void shard_sumsq_add(const float* g, const ShardRanges& r, float* partials, float* out, OptScalars* sc, hipStream_t st);
struct PnormParts {  // [0] critic, [1] actor
  const float* pt[2]; int nt[2];
  const float* ph[2]; int nh[2];
  OptScalars* sc[2];
};

struct AlphaParams {
  const float* logpi;   // [B] (actor pass)
  const int* counts;    // per local task
  const int* rows;
  int max_rows;
  int T_l, task_begin, T_glob, B_glob;
  float target_entropy;
  float* log_alpha;     // [T_glob] replicated
  float* m; float* v;
  float* grad;          // [T_glob] scratch (allreduced in multi-GPU)
  float* loss_part;     // scalar scratch: sum over rows of -(log_alpha_t)(logpi + H)
  float* task_loss;     // [T_glob] scratch: that sum per task
  OptScalars* sc;
};
// grad[t], task_loss[t] and *loss_part (one launch)
void alpha_grad(const AlphaParams& a, hipStream_t st);

struct LogParams {
  const float* critic_sums;  // [0] sum w (q - y)^2 over members, [1] sum q
  const float* actor_sums;   // [0] sum of actor loss terms
  const OptScalars* critic; const OptScalars* actor;
  const float* alpha_loss_sum;
  const float* log_alpha; int T_glob;
  float inv_critic; float inv_actor; float inv_b;
  float* logs;
};

// The step's scalar tail, one launch: *row_out[k] = sum rows[k][0..B) for the non-null rows[k]
// (reduce_rows' order); the temperature Adam; sc[w]->pnorm = sqrt(sum pt[w] + (head_sq ?
// head_sq[w] : sum ph[w])); the logs; *counter += 1
// split2h: the optimizer's per-block weight maxima into the weight records (blocks [0, nh) of a
// params job cover the heads -> amax[1], the rest the trunk -> amax[0]; a target job (nh < 0) -> amax[0])
struct WeightMaxJob {
  const float* parts; int n, nh;
  PlaneRec* rec;
};
struct StepFinish {
  const float* rows[3]; float* row_out[3]; int B;
  AlphaParams alpha; int alpha_grad;  // alpha_grad: also the temperature gradient (alpha_grad's work) first
  float lr, b1, b2, eps, max_norm;
  PnormParts pn; const float* head_sq;
  LogParams logs;
  unsigned long long* counter;
  WeightMaxJob wmax[3]; int nwmax;
};
void step_finish(const StepFinish& f, hipStream_t st);
// split2h: a weight record from the parameters as they lie (set_params): maxima and the planes' exponent
void weights_record(const float* p, long long trunk_off, long long n_flat, PlaneRec* rec, hipStream_t st);

// ------------------------------------------------------------------ gradient-conflict statistics
// (conflict.hip; MTSAC.compute_weights, mtsac.py:733-1170 and algorithms/utils.py:49-174)
// G: per-task gradients [T][P] (flax ravel order, T <= 64).  values[t*2 + k] = the ranks[t*2 + k]-th
// smallest |G[t][:]| (0-based); blocking (returns to the host).
void task_select(const float* G, int T, long long P, const long long* ranks, float* values, unsigned* ws_prefix,
                 long long* ws_rank, unsigned* ws_hist, hipStream_t st);
// one pass over G: gram[64*64] (fp64), l1[64], counts[4][64*64] = #(g_i g_j < 0), #(S_i & S_j),
// #(S_i & S_j & g_i g_j < 0), #(|g_i| < eps & |g_j| > tau) with S_t = |g_t| >= thr[t]; nz[t] = #(|g_t| < eps)
void task_pair_stats(const float* G, int T, long long P, const float* thr, float eps, float tau, int grid,
                     double* ws_gram_part, double* ws_l1_part, unsigned long long* counts, unsigned long long* nz,
                     double* gram, double* l1, hipStream_t st);
// dst[t*P + dst_off + e*dst_ms + t*blk + i] = src[src_off + e*src_ms + t*blk + i], i < blk (per-task head blocks)
void scatter_task_blocks(const float* src, long long src_off, long long src_ms, float* dst, long long P,
                         long long dst_off, long long dst_ms, int E, int T, long long blk, hipStream_t st);
// *err |= 1 unless task[r] == r % T_l for every row (rows interleaved i*T + t, as the buffer samples)
void check_interleaved(const int* task, int B, int T_l, int* err, hipStream_t st);

}  // namespace mtsac
