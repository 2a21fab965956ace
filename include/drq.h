/* drq.h -- C ABI of the MI355X DrQ-eps update engine (libmtsac.so), SURVEY.md section 8(f) row 4.
 *
 * Replaces, for experiments/atari.py's multi-task Atari agent, the device part of
 *   DrQ.update / DrQ._update_inner   (mtrl/rl/algorithms/drqeps.py:268-335, 337-343):
 *   augment (mtrl/nn/augmentation.py:101-117) of obs and next_obs, the online and target
 *   ImpalaDQN forwards at s' (greedy a*, C51 projection of the target distribution), the online
 *   forward + backward at s (cross entropy at the taken action), optax.adamw (lr, eps, weight
 *   decay; no clip) and the Polyak target, with the same LogDict.
 * The network is ImpalaDQN (mtrl/rl/networks.py:127-149): IMPALA encoder (stacks 8/16/16 x scale,
 * 2 residual blocks each, mtrl/nn/impala.py:13-48) ++ unit-norm task embedding, LayerNorm,
 * DistributionalDense (Dense 512 x scale, LayerNorm, ReLU, dueling adv/value over n_atoms).
 *
 * Conventions (as include/mtsac.h): plain pointers and sizes, negative errno on failure with
 * drq_last_error(), the engine owns device memory, one engine per GPU, all work on its stream.
 * Parameter vectors cross the boundary as ONE flat float array in flax ravel_pytree order (dict
 * keys sorted at every level), the same order oracle/drq.py's param_spec() lists.
 * The reference draws the augmentation's crop offsets and intensity factors from jax.random
 * (threefry, not reproduced): they are inputs here.
 */
#ifndef MTSAC_DRQ_H
#define MTSAC_DRQ_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct drq_config {
  int num_tasks;    /* 26 (experiments/atari.py:31) */
  int n_actions;    /* 18 (ALE full action set) */
  int n_atoms;      /* 51 (ImpalaDQN.num_atoms default; the config's 101 is not passed through) */
  int in_ch;        /* 4 stacked frames */
  int hw;           /* 84 */
  int scale;        /* ImpalaEncoderConfig.scale (atari.py Args.scale = 1) */
  int embed_dim;    /* 32 */
  int n_hidden;     /* 512 (times scale) */
  int batch;        /* samples per update (DrQTrainingConfig.batch_size = 256) */
  int nstep;        /* 3 */
  float gamma, v_min, v_max, tau;                 /* 0.99, -10, 10, 0.005 */
  float lr, b1, b2, eps, weight_decay, ln_eps;    /* 1e-4, 0.9, 0.999, 1.5e-4, 0.05, 1e-6 */
  long long capacity;     /* replay slots per task (0: no device buffer; buffer_size / num_tasks) */
  int normalize_rewards;  /* per-task min-max reward normalisation at sample time */
  int buffer_kind;        /* DRQ_BUFFER_MEMORY_EFFICIENT (0) or DRQ_BUFFER_ATARI (1) */
} drq_config;

/* MemoryEfficientAtariMultiTaskReplayBuffer (buffers.py:949-1279): next_obs is the slot nstep
 * ahead in the one frame array, indices avoid the guard window [pos, pos + nstep + 6). */
#define DRQ_BUFFER_MEMORY_EFFICIENT 0
/* AtariMultiTaskReplayBuffer (buffers.py:710-947): a second frame array for next_obs, indices in
 * [0, max(pos or capacity, n)) with no guard window. */
#define DRQ_BUFFER_ATARI 1

typedef struct drq_engine drq_engine;

/* One update's inputs (host or device pointers): observations uint8 [batch][in_ch][hw][hw]
 * (NCHW, as the Atari buffer stores them), actions int [batch], rewards / dones float [batch]
 * (n-step returns and terminal flags), task ids int [batch], and the augmentation draws:
 * crop offsets int [batch][2] in [0, 8) and intensity factors float [batch] for obs and next_obs. */
typedef struct drq_batch {
  const unsigned char* obs;
  const int* actions;
  const unsigned char* next_obs;
  const float* dones;
  const float* rewards;
  const int* task_ids;
  const int* crop_obs;
  const float* noise_obs;
  const int* crop_next;
  const float* noise_next;
} drq_batch;

#define DRQ_PARAMS 0
#define DRQ_TARGET 1
#define DRQ_ADAM_MU 2
#define DRQ_ADAM_NU 3
#define DRQ_GRAD 4 /* the last update's gradient (get only) */
#define DRQ_NUM_LOGS 4 /* losses/online_logits, metrics/critic_grad_magnitude,
                          metrics/critic_params_norm, losses/critic_loss (drqeps.py:309-335) */

int drq_create(const drq_config* cfg, int device, drq_engine** out);
void drq_destroy(drq_engine* e);
long long drq_num_params(const drq_engine* e);
/* which: DRQ_PARAMS / DRQ_TARGET / DRQ_ADAM_MU / DRQ_ADAM_NU (/ DRQ_GRAD for get); n = drq_num_params */
int drq_set_params(drq_engine* e, int which, const float* flat, long long n);
int drq_get_params(drq_engine* e, int which, float* flat, long long n);
int drq_set_step(drq_engine* e, int adam_count);
/* the AdamW step count (optax ScaleByAdamState.count): bias correction of the next update */
int drq_get_step(drq_engine* e, int* adam_count);
/* stage one batch and run one update on it (asynchronous on the engine's stream) */
int drq_update(drq_engine* e, const drq_batch* batch);
/* run `steps` more updates on the batch already resident on the device (benchmarks), each with
 * fresh device augmentation draws */
int drq_update_resident(drq_engine* e, int steps);
/* expected Q [n][n_actions] of the online network on n <= batch observations (uint8 NCHW), after
 * the augmentation with the given draws: the quantity _sample_action / _eval_action take the argmax
 * of (drqeps.py:56-97); epsilon-greedy stays with the caller's RNG.  Synchronous. */
int drq_q_values(drq_engine* e, const unsigned char* obs, const int* task_ids, const int* crop, const float* noise,
                 int n, float* q);
/* The device replay buffer, MemoryEfficientAtariMultiTaskReplayBuffer (mtrl/rl/buffers.py:949-1229):
 * one uint8 frame-stack array [capacity][num_tasks][in_ch][hw][hw] holds obs and next_obs (nstep
 * slots ahead).  add: one env step of all tasks (host pointers; the n-step ring runs on the host
 * exactly as buffers.py:1048-1186 does).  The index stream is numpy's Generator (PCG64) whose state
 * drq_rng_set takes (bit_generator.state), reproduced bit for bit on the device. */
int drq_buffer_add(drq_engine* e, const unsigned char* obs, const unsigned char* next_obs, const int* action,
                   const float* reward, const float* truncate, const float* done);
int drq_buffer_state(drq_engine* e, long long* pos, int* full);
int drq_rng_set(drq_engine* e, unsigned long long state_hi, unsigned long long state_lo, unsigned long long inc_hi,
                unsigned long long inc_lo, int has_uint32, unsigned int uinteger);
/* sample(batch) from the device buffer into the engine's staged batch (batch % num_tasks == 0) */
int drq_sample(drq_engine* e);
/* `steps` x (sample + update): DrQ's training step with the batch drawn on the device (the
 * augmentation crops / intensities from the device counter hash seeded by drq_seed_augment) */
int drq_sample_update(drq_engine* e, int steps);
/* sample_unbalanced (buffers.py:1230-1279, what OffPolicyAlgorithm.train calls for this buffer,
 * base.py:217-218): the caller draws the Dirichlet task sizes and the per-task slots with its own
 * Generator and passes `batch` rows (slot in [0, capacity), task id in [0, num_tasks)); the gather,
 * next_obs nstep ahead and the reward normalisation run on the device. */
int drq_sample_rows(drq_engine* e, const long long* slots, const int* task_ids);
/* `steps` x (sample_rows + update) on [steps][batch] host-drawn rows */
int drq_sample_rows_update(drq_engine* e, const long long* slots, const int* task_ids, int steps);
/* the device PCG64 state after drq_sample: state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger */
int drq_rng_get(drq_engine* e, unsigned long long* out6);
int drq_seed_augment(drq_engine* e, unsigned long long seed);
/* the staged batch (tests): uint8 obs / next_obs, actions, rewards, dones, truncations, task ids */
int drq_read_batch(drq_engine* e, unsigned char* obs, unsigned char* next_obs, int* actions, float* rewards,
                   float* dones, float* truncations, int* task_ids);
int drq_get_logs(drq_engine* e, float* out /* DRQ_NUM_LOGS */);
/* compute_weights (drqeps.py:353-482).  drq_task_gradient: the loss gradient (no optimizer step)
 * of one task group's `batch` rows, stored in flax ravel order as row `slot` of the engine's
 * per-task gradient matrix [num_slots][drq_num_params] (grown on demand).
 * drq_project_task_gradients: project_grad (drqeps.py:428-448) of the first num_slots rows,
 * out[t][j] = sum_k g_t[k] N(k, j) / sqrt(proj_dim), N the (chunk x proj_dim) blocks of
 * jax.random.normal(PRNGKey(seed + block)) regenerated on the device (threefry2x32, jax 0.5.3
 * partitionable bits); out is host or device, [num_slots][proj_dim].  Synchronous. */
int drq_task_gradient(drq_engine* e, const drq_batch* batch, int slot, int num_slots);
int drq_get_task_gradient(drq_engine* e, int slot, float* flat, long long n);
int drq_project_task_gradients(drq_engine* e, int num_slots, int proj_dim, long long chunk, int seed, float* out);
int drq_synchronize(drq_engine* e);
/* bench.py's roofline: HIP events around the IMPALA conv forward launches of every 8th update on
 * the engine stream while on; drq_timing sums them (ms), with the launch count and algorithmic flops 2 B H W 9 ci co */
int drq_set_timing(drq_engine* e, int on);
int drq_timing(drq_engine* e, double* ms, long long* launches, double* flops);
const char* drq_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
