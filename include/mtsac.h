/*
 * mtsac.h -- C-ABI of the MI355X multi-task SAC update engine (libmtsac.so).
 *
 * Drop-in boundary for the reference's MTSAC hot path.  Every entry point
 * cites the reference interface it replaces (paths relative to the
 * reginald-mclean/mtrl tree):
 *
 *   mtsac_create / mtsac_destroy   MTSAC.initialize      mtrl/rl/algorithms/mtsac.py:153-284
 *                                  (device state instead of a flax PyTree)
 *   mtsac_set_params/get_params    TrainState params / opt_state leaves
 *                                  mtrl/rl/algorithms/utils.py:11-46, mtsac.py:197-256
 *   mtsac_buffer_add[_stream]      MultiTaskReplayBuffer.add        mtrl/rl/buffers.py:426-474
 *   mtsac_buffer_write             MultiTaskReplayBuffer.load_checkpoint data  buffers.py:326-335
 *   mtsac_buffer_read              MultiTaskReplayBuffer.checkpoint data       buffers.py:308-324
 *   mtsac_buffer_set/get_state     pos / full fields                buffers.py:306,337-343
 *   mtsac_rng_set / mtsac_rng_get  buffer _rng PCG64 state          buffers.py:260,323,335
 *   mtsac_sample                   MultiTaskReplayBuffer.sample(int) buffers.py:494-549
 *   mtsac_update                   MTSAC.update -> _update_inner     mtsac.py:1173-1251
 *   mtsac_get_logs                 the update's LogDict              mtsac.py:1241-1247
 *   mtsac_eval_action              MTSAC.eval_action / _eval_action  mtsac.py:80-84,306-311
 *   mtsac_sample_action            MTSAC.sample_action               mtsac.py:70-77,298-304
 *   mtsac_comm_*                   (new) task-sharded data parallelism over RCCL; the
 *                                  reference is single-device
 *
 * Conventions
 *   - Return value: 0 on success, a negative errno-style code on failure; the
 *     thread-local message is available from mtsac_last_error().  Nothing aborts.
 *   - The engine owns all device memory.  Callers own every pointer they pass;
 *     pointers are borrowed for the duration of the call only.  Data pointers may
 *     be host or device (HIP unified addressing: hipMemcpyDefault).
 *   - One engine per GPU per process.  All work of an engine is serialised on its
 *     own HIP stream; mtsac_get_logs / mtsac_sample / mtsac_get_params are the
 *     synchronisation points.
 *   - Parameter vectors use the flax leaf order (ravel_pytree order) of the
 *     reference networks: head bias, head kernel, layer_0 bias, layer_0 kernel,
 *     layer_1 ... (critic leaves carry the leading ensemble axis).  With task
 *     sharding (task_count < num_tasks) the head leaves hold only the local tasks.
 */
#ifndef MTSAC_H_
#define MTSAC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTSAC_ABI_VERSION 1
#define MTSAC_NUM_LOGS 10

/* log slots, order of mtsac.py:1241-1247 (critic, actor, alpha logs) */
enum mtsac_log_slot {
  MTSAC_LOG_QF_VALUES = 0,          /* losses/qf_values                */
  MTSAC_LOG_QF_LOSS = 1,            /* losses/qf_loss                  */
  MTSAC_LOG_CRITIC_GRAD_NORM = 2,   /* metrics/critic_grad_magnitude   */
  MTSAC_LOG_CRITIC_PARAMS_NORM = 3, /* metrics/critic_params_norm      */
  MTSAC_LOG_ACTOR_LOSS = 4,         /* losses/actor_loss               */
  MTSAC_LOG_ACTOR_GRAD_NORM = 5,    /* metrics/actor_grad_magnitude    */
  MTSAC_LOG_ACTOR_PARAMS_NORM = 6,  /* metrics/actor_params_norm       */
  MTSAC_LOG_EXPLORE_LOSS = 7,       /* metrics/explore_loss (always 0) */
  MTSAC_LOG_ALPHA_LOSS = 8,         /* losses/alpha_loss               */
  MTSAC_LOG_ALPHA = 9               /* alpha = sum(exp(log_alpha))     */
};

/* which parameter / optimizer vector mtsac_{get,set}_params addresses */
enum mtsac_tensor {
  MTSAC_ACTOR = 0,
  MTSAC_CRITIC = 1,
  MTSAC_CRITIC_TARGET = 2,
  MTSAC_LOG_ALPHA_PARAMS = 3,
  MTSAC_ACTOR_ADAM_MU = 4,
  MTSAC_ACTOR_ADAM_NU = 5,
  MTSAC_CRITIC_ADAM_MU = 6,
  MTSAC_CRITIC_ADAM_NU = 7,
  MTSAC_ALPHA_ADAM_MU = 8,
  MTSAC_ALPHA_ADAM_NU = 9
};

enum mtsac_precision {
  MTSAC_FP32 = 0,       /* f32-input MFMA (v_mfma_f32_32x32x2_f32), fp32 everywhere          */
  MTSAC_FP32_SPLIT3 = 1, /* fp32-accurate trunk GEMMs on bf16 MFMA: each fp32 operand split
                           exactly into 3 bf16 terms, 6 cross products accumulated in fp32
                           (dropped terms <= 2^-23 relative); everything else fp32           */
  MTSAC_BF16 = 2,        /* perf-only: the trunk GEMMs' operands rounded to bf16 (the high
                           term of the same split), one bf16 MFMA per product, fp32
                           accumulation; master weights, Adam, heads, losses stay fp32.
                           NOT the reference's arithmetic (fp32): losses drift ~1e-3 rel  */
  MTSAC_FP32_SPLIT2H = 3 /* fp32-accurate trunk GEMMs on fp16 MFMA: each operand tensor scaled
                           by a power of two 2^e (per tensor, from an a-priori bound of its
                           values) and split into 2 fp16 terms (22 significant bits),
                           3 cross products (h*l, l*h, h*h) accumulated in fp32, unscaled
                           exactly; same GEMM error bound as split3 (<= 4e-6 sum|a b|)      */
};

/* Hyper-parameters: MTSACConfig (mtsac.py:116-127) + AlgorithmConfig
 * (config/rl.py:16-22) + ContinuousActionPolicyConfig / QValueFunctionConfig
 * (config/networks.py:6-31) + MultiHeadConfig (config/nn.py:8-31,63) +
 * OptimizerConfig (config/optim.py:14-43) + OffPolicyTrainingConfig
 * (config/rl.py:47-50). */
typedef struct mtsac_config {
  int32_t num_tasks;        /* T: width of the one-hot at the end of obs       */
  int32_t task_begin;       /* first task owned by this engine (sharding)      */
  int32_t task_count;       /* tasks owned by this engine (= T unsharded)      */
  int32_t obs_dim;          /* observation width incl. one-hot (39 + T)        */
  int32_t action_dim;       /* A (4)                                           */
  int32_t actor_width, actor_depth;
  int32_t critic_width, critic_depth;
  int32_t num_critics;      /* ensemble size (2)                               */
  int32_t batch_per_task;   /* B / T (128)                                     */
  int64_t capacity;         /* slots per task = buffer_size // T               */
  float gamma, tau;
  float actor_lr, critic_lr, alpha_lr;
  float actor_max_grad_norm, critic_max_grad_norm, alpha_max_grad_norm; /* < 0 (None): no
                               clip; >= 0: optax clip_by_global_norm, 0 included (config/optim.py:38) */
  float adam_b1, adam_b2, adam_eps;
  float initial_temperature;
  float log_std_min, log_std_max;
  int32_t clip;             /* clip y and Q to +-5000 (mtsac.py:557-560)        */
  int32_t use_task_weights; /* mtsac.py:103-113                                 */
  int32_t normalize_rewards;/* 0 off, 1 per-task min/max (buffers.py:534-538), 2 return
                               normalisation (buffers.py:392-422, 531-533): rewards divided
                               by the per-task denominator the host sets through
                               mtsac_buffer_set_reward_stats(min = 0, max = denominator) */
  int32_t precision;        /* enum mtsac_precision                             */
  uint64_t noise_seed;      /* device N(0,1) stream used when no eps is injected */
} mtsac_config;

/* A batch laid out like ReplayBufferSamples (types.py:49-54): rows of this
 * engine's tasks, row = i * task_count + local_task. */
typedef struct mtsac_batch {
  const float* observations;      /* [B_local][obs_dim]    */
  const float* actions;           /* [B_local][action_dim] */
  const float* next_observations; /* [B_local][obs_dim]    */
  const float* dones;             /* [B_local]             */
  const float* rewards;           /* [B_local]             */
} mtsac_batch;

typedef struct mtsac_engine mtsac_engine;

const char* mtsac_last_error(void);
int mtsac_abi_version(void);
/* Build provenance: the first 16 hex digits of the sha256 of the sources the library was built from
 * (the .hip, .cpp and .h files of mtrl_amd/csrc and the .h files of include, in sorted relative-path
 * order, concatenated; mtrl_amd/csrc/Makefile). */
const char* mtsac_build_stamp(void);
void mtsac_default_config(mtsac_config* cfg, int32_t num_tasks);

int mtsac_create(const mtsac_config* cfg, int hip_device, mtsac_engine** out);
void mtsac_destroy(mtsac_engine* h);

/* parameters / optimizer state, flax leaf order, fp32 */
int64_t mtsac_param_count(const mtsac_engine* h, int which);
int mtsac_set_params(mtsac_engine* h, int which, const float* src, int64_t n);
int mtsac_get_params(mtsac_engine* h, int which, float* dst, int64_t n);
int mtsac_set_adam_count(mtsac_engine* h, int which /*0 actor,1 critic,2 alpha*/, int32_t count);
int mtsac_get_adam_count(mtsac_engine* h, int which, int32_t* count);

/* replay buffer (device resident; layout documented in DESIGN.md).
 * buffer_add (buffers.py:426-474) does not block the host: the T_local rows are staged through
 * a pinned ring and written + committed on the engine stream, ordered after every update issued
 * before it and before every update issued after it.  Pass the five arrays all in host memory
 * or all in device memory.  Device arrays are read after the work already queued on the
 * producer stream (mtsac_buffer_add: the legacy default stream; mtsac_buffer_add_stream: the
 * hipStream_t passed as producer_stream, e.g. torch.cuda.current_stream().cuda_stream), and
 * the producer stream is made to wait for that read, so the caller may free or overwrite the
 * arrays right after the call.  Reward min / max (normalize_rewards) are kept on the device. */
int mtsac_buffer_add(mtsac_engine* h, const float* obs, const float* next_obs, const float* actions,
                     const float* rewards, const float* dones);
int mtsac_buffer_add_stream(mtsac_engine* h, const float* obs, const float* next_obs, const float* actions,
                            const float* rewards, const float* dones, void* producer_stream);
int mtsac_buffer_write(mtsac_engine* h, int64_t slot_begin, int64_t n_slots, const float* obs,
                       const float* next_obs, const float* actions, const float* rewards,
                       const float* dones);
int mtsac_buffer_read(mtsac_engine* h, int64_t slot_begin, int64_t n_slots, float* obs, float* next_obs,
                      float* actions, float* rewards, float* dones);
int mtsac_buffer_fill_synthetic(mtsac_engine* h, uint64_t seed);
int mtsac_buffer_set_state(mtsac_engine* h, int64_t pos, int32_t full);
int mtsac_buffer_get_state(mtsac_engine* h, int64_t* pos, int32_t* full);
/* normalize_rewards 1: the running per-task reward min / max; 2: (0, denominator) */
int mtsac_buffer_set_reward_stats(mtsac_engine* h, const double* min_r, const double* max_r);
int mtsac_buffer_get_reward_stats(mtsac_engine* h, double* min_r, double* max_r);
int mtsac_rng_set(mtsac_engine* h, uint64_t state_hi, uint64_t state_lo, uint64_t inc_hi,
                  uint64_t inc_lo, int32_t has_uint32, uint32_t uinteger);
int mtsac_rng_get(mtsac_engine* h, uint64_t* state_hi, uint64_t* state_lo, uint64_t* inc_hi,
                  uint64_t* inc_lo, int32_t* has_uint32, uint32_t* uinteger);
/* draw one batch with the device index stream and copy it (and the indices) out */
int mtsac_sample(mtsac_engine* h, int64_t* indices, float* obs, float* actions, float* next_obs,
                 float* dones, float* rewards);

/* one gradient step.  batch == NULL: sample from the device buffer.
 * eps_next / eps_cur ([B_local][A] N(0,1) noise for a' ~ pi(.|s') and a ~ pi(.|s));
 * both NULL: device counter-based normal stream. */
int mtsac_update(mtsac_engine* h, const mtsac_batch* batch, const float* eps_next, const float* eps_cur);
/* run `steps` device-sampled, device-noise updates (hipGraph replay when enabled) */
int mtsac_update_many(mtsac_engine* h, int32_t steps);
int mtsac_get_logs(mtsac_engine* h, float* logs /* MTSAC_NUM_LOGS */);
int mtsac_enable_graph(mtsac_engine* h, int32_t enable);
int mtsac_synchronize(mtsac_engine* h);

/* rollout side */
int mtsac_eval_action(mtsac_engine* h, const float* obs, int32_t n, float* actions);
int mtsac_sample_action(mtsac_engine* h, const float* obs, int32_t n, const float* eps, float* actions);

/* multi-GPU: RCCL communicator over the shared-trunk gradients */
int mtsac_comm_unique_id_size(void);
int mtsac_comm_get_unique_id(void* id_out);
/* mtsac_comm_init waits for every peer (MTSAC_COMM_INIT_TIMEOUT_S in the environment bounds the
 * wait); mtsac_comm_init_timeout returns -110 (ETIMEDOUT) when the peers have not joined within
 * timeout_s seconds (<= 0: wait forever) and leaves the engine without a communicator. */
int mtsac_comm_init(mtsac_engine* h, const void* unique_id, int32_t nranks, int32_t rank);
int mtsac_comm_init_timeout(mtsac_engine* h, const void* unique_id, int32_t nranks, int32_t rank,
                            double timeout_s);
/* device noise stream (used when no eps is injected): seed and step counter; setting them
 * rebuilds the step graph (checkpoint / resume of the update noise) */
int mtsac_get_noise_state(mtsac_engine* h, uint64_t* seed, uint64_t* counter);
int mtsac_set_noise_state(mtsac_engine* h, uint64_t seed, uint64_t counter);
/* ranks in the engine's communicator as RCCL reports them (ncclCommCount); 1 without one */
int mtsac_comm_nranks(mtsac_engine* h, int32_t* nranks);
/* Bring-your-own collective: when no RCCL communicator is set, the engine calls
 * fn(user, device_buffer, count) at each all-reduce point (after synchronising its
 * stream), at the same points and in the same order as the RCCL path: one bucket per hidden
 * layer as its weight gradient completes, then layer 0 and the scalar tail; fn must leave the
 * element-wise SUM over all shards in the buffer (completed on the device) before returning.
 * Disables hipGraph replay for this engine.  fn == NULL removes it. */
typedef int (*mtsac_allreduce_fn)(void* user, float* device_buffer, int64_t count);
int mtsac_set_allreduce_hook(mtsac_engine* h, mtsac_allreduce_fn fn, void* user);
/* The same with the sharded optimizer's collectives too: fn(user, op, device_buffer, count), op 0 =
 * all-reduce (sum), 1 = reduce-scatter in place (rank r's shard [r count / world, (r + 1) count / world)
 * of the buffer must hold the element-wise sum over all ranks; the rest is left undefined), 2 =
 * all-gather in place (every rank's shard of the buffer from its owner).  rank / world: this engine's
 * place in the group.  Replaces an all-reduce hook; fn == NULL removes it. */
typedef int (*mtsac_collective_fn)(void* user, int32_t op, float* device_buffer, int64_t count);
int mtsac_set_collective_hook(mtsac_engine* h, mtsac_collective_fn fn, void* user, int32_t rank, int32_t world);
/* Sharded trunk optimizer (ZeRO-1 style) for task-sharded runs (reference OptimizerConfig.spawn /
 * TrainState.apply_gradients, mtrl/config/optim.py:26-43, mtrl/rl/algorithms/utils.py:11-46): every trunk
 * bucket is reduce-scattered instead of all-reduced, the global clip norm comes from an all-reduced
 * |g|^2, each rank runs Adam on its 1/world of the trunk, the new trunk is all-gathered and every
 * rank writes its own GEMM planes and Polyak target from it.  on: 1 / 0; active only with an RCCL
 * communicator or a collective hook (not the one-GPU modelled collective, whose collectives move no data),
 * with world > 1, at most 7 trunk buckets and world dividing every bucket into whole float4s (else the
 * all-reduce path runs).  Switching drops a captured step graph.  The Adam moments then live sharded:
 * get_params of a moment returns this rank's shards current, the rest stale.  Default off (MTSAC_ZERO=1
 * turns it on). */
int mtsac_set_sharded_optimizer(mtsac_engine* h, int32_t on);
/* plain device/host copy helper for hooks written in a host language (hipMemcpyDefault) */
int mtsac_memcpy(void* dst, const void* src, int64_t bytes);

/* measurement: per-kernel-family HIP event timing (events on each launch's own stream) over all
 * steps of the last update / update_many call.  enable: 0 off, 1 on (the step keeps its
 * concurrent streams; forces eager issue), 2 on with every kernel serialised on one stream (solo
 * kernel durations).  Families (enum mtsac_gemm_family):
 * hidden-layer forward, hidden-layer data grad, hidden-layer weight grad, input-layer forward,
 * input-layer weight grad. */
enum mtsac_gemm_family {
  MTSAC_FAM_FORWARD = 0,
  MTSAC_FAM_DATA_GRAD = 1,
  MTSAC_FAM_WEIGHT_GRAD = 2,
  MTSAC_FAM_INPUT_FORWARD = 3,
  MTSAC_FAM_INPUT_WEIGHT_GRAD = 4
};
int mtsac_set_timing(mtsac_engine* h, int32_t enable);
int mtsac_get_timing(mtsac_engine* h, int32_t family, double* total_ms, int32_t* launches,
                     double* flops);
/* the kernel behind a GEMM family at its last launch (labels for the bench and profiles) */
int mtsac_get_timing_kernel(mtsac_engine* h, int32_t family, char* buf, int32_t n);

/* ---- eval-time gradient-conflict statistics (MTSAC.compute_weights, mtsac.py:870-1170;
 * compute_gram_metrics :733-771, compute_support_metrics :774-867; vmap_cos_sim /
 * compute_conflict_metrics, algorithms/utils.py:49-174).  Unsharded engines only (-95).
 * mtsac_task_gradients: per-task gradients of each task's own loss (critic MSE over its n rows,
 * actor loss over its rows) on the CURRENT parameters, into device matrices [T][P] in flax ravel
 * order (which 0 = critic, P = mtsac_task_gradient_size(h, 0); 1 = actor).  batch NULL = sample
 * on device; rows must be interleaved i*T + t (as MultiTaskReplayBuffer.sample returns them).
 * eps_next (the reference samples these from pi(.|s), mtsac.py:1000-1004) / eps_cur: [B][A]
 * injected noise, or both NULL (device noise).  Nothing is updated.
 * mtsac_task_gradient_select: values[t*2+k] = the ranks[t*2+k]-th smallest |g_t| (0-based),
 * the two order statistics of jnp.quantile's linear interpolation.
 * mtsac_task_gradient_stats: one pass over G with support S_t = |g_t| >= thresholds[t]:
 * gram[T*T] = G G^T, l1[T] = sum |g_t|, counts[4][T*T] = #(g_i g_j < 0), #(S_i & S_j),
 * #(S_i & S_j & g_i g_j < 0), #(|g_i| < eps & |g_j| > tau); near_zero[T] = #(|g_t| < eps).
 * The T x T algebra on top is host code (mtrl_amd/conflict.py). */
int mtsac_task_gradients(mtsac_engine* h, const mtsac_batch* batch, const float* eps_next,
                         const float* eps_cur);
int64_t mtsac_task_gradient_size(const mtsac_engine* h, int which);
int mtsac_get_task_gradients(mtsac_engine* h, int which, float* dst, int64_t n);
int mtsac_set_task_gradients(mtsac_engine* h, int which, const float* src, int64_t n);
int mtsac_task_gradient_select(mtsac_engine* h, int which, const int64_t* ranks, float* values);
int mtsac_task_gradient_stats(mtsac_engine* h, int which, const float* thresholds, float eps,
                              float tau, double* gram, double* l1, int64_t* counts,
                              int64_t* near_zero);

#ifdef __cplusplus
}
#endif
#endif /* MTSAC_H_ */
