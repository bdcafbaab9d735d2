/*
 * ballbot_mi355x.h -- C-ABI drop-in boundary for the batched ballbot hot path.
 *
 * Replaces, for N envs at once on one MI355X, what the reference does per env
 * through MuJoCo's pybind11 API inside BBotSimulation:
 *   bb_create        mujoco.MjModel.from_xml_path + MjData      ballbot_env.py:261-262
 *   bb_set_hfield    model.hfield_data = terrain_gen(n, seed)   ballbot_env.py:513
 *                    (+ hfield_size[2] rescale                  ballbot_env.py:486-495)
 *                    (+ init height offset                      ballbot_env.py:527-565)
 *   bb_generate_perlin  generate_perlin_terrain per seed       terrain/perlin.py:8-74
 *   bb_set_terrain_rng     r_seed = _np_random.integers(0, 10000) ballbot_env.py:505-510,
 *                    at every reset, numpy's PCG64 per env on the    :378-384, 596 (SB3 reset(seed=seed+i),
 *                    GPU (gymnasium np_random)                       train.py:82-97, 126-141)
 *   bb_set_terrain_stream  the same draws as a host-made table   ballbot_env.py:505-510
 *   bb_assign_terrain   pin a terrain per env (config seed)     ballbot_env.py:505-510
 *   bb_reset         mj_resetData + height offset + mj_forward  ballbot_env.py:612-620
 *   bb_step          ctrl = -clip(10a); mj_step; _get_obs;      ballbot_env.py:903-1036
 *                    reward plugin; termination
 *   bb_render_depth  RGBDInputs depth cams (_get_obs)           sensors/rgbd.py:46-82
 *   bb_ppo_loss      SB3 PPO.train minibatch loss + grads
 *   bb_adamw_clip    SB3 PPO.train clip_grad_norm_ + AdamW step
 *   bb_ppo_mlp_step  SB3 PPO.train minibatch (forward, loss, backward, clip,
 *                    AdamW) of the reference's proprio MLP policy, fused
 *   bb_ppo_mlp_act   SB3 collect_rollouts policy step (same policy)
 *   bb_rollout_track SB3 collect_rollouts / Monitor episode bookkeeping
 *   bb_rollout       a whole SB3 collect_rollouts (policy + step + bookkeeping) in one launch
 *   bb_depth_encoder frozen rgbd encoder of the camera policy, fused
 *   bb_gae           SB3 RolloutBuffer.compute_returns_and_advantage (PPO)
 *   bb_forward       mujoco.mj_forward (diagnostic)             ballbot_env.py:525,620
 *   bb_get_state/    read/write qpos/qvel/qacc_warmstart        ballbot_env.py:616-617
 *   bb_set_state     (MjData.qpos / qvel)
 *
 * Conventions
 *   - every function returns int: 0 ok, <0 error (bb_last_error has the text);
 *     per-env physics divergence is NOT an error.  As MuJoCo's mj_step does
 *     (mj_checkPos/Vel at its start, mj_checkAcc after the first forward), a
 *     NaN or |x| > 1e10 in qpos, qvel or qacc resets that env's data to qpos0
 *     (no terrain height offset, zero velocity, warm start and ctrl) and the
 *     step integrates from there; the episode goes on (no done), done[] bit 2
 *     reports it.  A NaN ctrl zeroes all three controls (mjWARN_BADCTRL).
 *   - device pointers belong to the caller (e.g. torch tensors); the library
 *     never frees them.  Work is enqueued on the caller's stream (hipStream_t
 *     passed as void*); bb_step/bb_reset are graph-capturable.
 *   - one handle per device; a handle is not thread-safe.
 *   - state layout (get/set): qpos[n][17], qvel[n][15], warm[n][15] in MuJoCo
 *     order (free joints: pos, quat(w,x,y,z); lin vel world, ang vel local).
 *   - obs layout [n][15]: sorted keys actions(3) angular_vel(3) motor_state(3)
 *     orientation(3) vel(3), the order the reference policy consumes.
 */
#ifndef BALLBOT_MI355X_H
#define BALLBOT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BB_ABI_VERSION 19
#define BB_NQ 17
#define BB_NV 15
#define BB_OBS 15
#define BB_HF_N 293

/* done[] bits (only TERMINATED ends an episode) */
#define BB_DONE_TERMINATED 1
#define BB_DONE_FAILURE 2
#define BB_DONE_DIVERGED 4 /* MuJoCo's divergence reset ran inside this step (informational) */
#define BB_DONE_OVERFLOW 8
#define BB_NSTATS 8
#define BB_NPAIR 19

/* reward kinds (built-in reward plugins, ballbot_gym/rewards) */
#define BB_REWARD_DIRECTIONAL 0 /* rewards/directional.py:33-54 */
#define BB_REWARD_DISTANCE 1    /* rewards/distance.py:33-50 (pos2d-based) */
#define BB_REWARD_NONE 2        /* custom plugin evaluated host-side: reward_dev gets the action penalty
                                   only; the caller adds plugin * scale, then the survival bonus when
                                   done bit 1 (failure) is clear (ballbot_env.py:929-937, 1019-1020) */

typedef struct bb_handle bb_handle;

/* BBotSimulation.__init__ settings (ballbot_env.py:157-231) */
typedef struct {
  int max_ep_steps;            /* 4000 */
  float max_allowed_tilt;      /* 20 degrees */
  float max_wheel_velocity;    /* 10 */
  float reward_scale;          /* 0.01 */
  float action_reg_coef;       /* -1e-4 */
  float survival_bonus;        /* 0.02 */
  float target_dir[2];         /* directional target (0, 1) */
  int reward_kind;             /* BB_REWARD_* */
  float goal[2];               /* distance reward goal */
  float goal_scale;            /* distance reward scale */
  int n_terrains;              /* terrain bank size (>= 1) */
  uint64_t seed;               /* unused since ABI 12 (terrain draws: bb_set_terrain_rng / _stream) */
  int fp64;                    /* 1 (default): fp64 arithmetic, 0: fp32 */
  int solver_maxiter;          /* 0 = default */
  double solver_tol;           /* 0 = default */
  /* mjModel.opt overrides (ABI 17; ballbot.xml:3-5): model.opt.timestep (0 = 0.002 s)
   * and disable flags with MuJoCo's mjtDisableBit values -- BB_DSBL_PASSIVE (joint
   * damping), BB_DSBL_GRAVITY.  For the physics invariants (tests/test_gpu_invariants.py);
   * the reference env never changes them. */
  double opt_timestep;
  int opt_disableflags;
} bb_params;
#define BB_DSBL_PASSIVE 32
#define BB_DSBL_GRAVITY 64

int bb_abi_version(void);
int bb_last_error(char* buf, int len);
void bb_default_params(bb_params* p);

int bb_create(int n_envs, int device, const bb_params* p, bb_handle** out);
int bb_destroy(bb_handle* h);

/* upload one terrain (host float32[293*293], row-major, values in [0,1]) */
int bb_set_hfield(bb_handle* h, int terrain_id, const float* data_host, float size_z);
/* perlin terrain generator arguments (terrain/perlin.py:8-16) */
typedef struct {
  double scale;       /* 25.0 */
  int octaves;        /* 4 */
  float persistence;  /* 0.2 */
  float lacunarity;   /* 2.0 */
  double amplitude;   /* 1.0 */
} bb_perlin_cfg;

/* generate perlin terrains for seeds_host[0..count) into bank slots
 * [first_terrain_id, first_terrain_id + count) on the GPU, with their init
 * offsets (synchronous).  Replaces generate_perlin_terrain(293, seed=s) +
 * the hfield_data write at reset (terrain/perlin.py:8-74, ballbot_env.py:501-513). */
int bb_generate_perlin(bb_handle* h, int first_terrain_id, int count, const int32_t* seeds_host,
                       const bb_perlin_cfg* cfg, float size_z);
/* PPO update boundary: GAE(gamma, lambda) advantages and returns of a device
 * rollout laid out [T][n_envs] (float32 rewards/values, uint8 episode starts;
 * last_values/last_dones [n_envs] for the bootstrap).  Replaces stable-
 * baselines3 RolloutBuffer.compute_returns_and_advantage as called by PPO
 * (ballbot_rl/training/train.py:125-142, model.learn at :284).  Enqueued on
 * stream; needs no handle. */
int bb_gae(const float* rewards_dev, const float* values_dev, const uint8_t* episode_starts_dev,
           const float* last_values_dev, const uint8_t* last_dones_dev, int T, int n_envs, double gamma,
           double gae_lambda, float* advantages_dev, float* returns_dev, void* stream);
/* depth cameras cam_0/cam_1 (ballbot.xml:44-54, fovy 90): for every env whose
 * step counter is a multiple of `every` (or all envs when force != 0), render
 * the linear z-depth clipped to 1 m into depth_dev float[n][2][height][width]
 * (row 0 = top); rel_ts_dev float[n] (may be NULL) receives
 * relative_image_timestamp = (steps % every) * 2 ms.  Replaces RGBDInputs with
 * disable_rgb (sensors/rgbd.py:46-82) as called by _get_obs
 * (ballbot_env.py:743-767, every = ceil((1/frame_rate)/dt), :389-411).
 * Enqueued on stream, after bb_step / bb_reset. */
int bb_render_depth(bb_handle* h, float* depth_dev, float* rel_ts_dev, int height, int width, int every,
                    int force, void* stream);
/* PPO update: fused minibatch loss of SB3 PPO.train (diagonal Gaussian,
 * clipped surrogate, MSE value loss, entropy; ppo/ppo.py, called through
 * model.learn at ballbot_rl/training/train.py:284) and its gradients.  All
 * pointers are device float32: mean/actions [B][3], values/old_logp/adv/
 * returns [B], log_std [3], clip (scalar).  Writes terms[9] = loss, pg, vf,
 * entropy loss, approx_kl, clip_fraction, dloss/dlog_std[3], grad_mean [B][3],
 * grad_values [B].  One workgroup, enqueued on stream; graph-capturable. */
int bb_ppo_loss(const float* mean_dev, const float* values_dev, const float* log_std_dev, const float* actions_dev,
                const float* old_logp_dev, const float* adv_dev, const float* returns_dev, const float* clip_dev,
                int B, int normalize_advantage, float ent_coef, float vf_coef, float* terms_dev,
                float* grad_mean_dev, float* grad_values_dev, void* stream);
/* SB3 PPO.train's optimiser step on flat fp32 device buffers of n elements:
 * clip_grad_norm_(max_norm) then torch.optim.AdamW (betas, eps, weight_decay;
 * learning rate read from lr_dev, step counter step_dev incremented on device;
 * coef_dev: 4 floats of scratch).  grad is read, not modified, and must be
 * 16-byte aligned.  Two launches on stream; graph-capturable.
 * Replaces SB3 2.6.0 PPO.train's clip_grad_norm_ + optimizer.step (the PPO the
 * reference builds in ballbot_rl/training/train.py:125-142). */
int bb_adamw_clip(float* param_dev, const float* grad_dev, float* exp_avg_dev, float* exp_avg_sq_dev, int64_t n,
                  const float* lr_dev, float* step_dev, float* coef_dev, double beta1, double beta2, double eps,
                  double weight_decay, double max_norm, void* stream);
/* One SB3 PPO.train minibatch of the reference's proprio policy, fused:
 * SB3 MultiInputPolicy with net_arch pi = vf = [128]*4, LeakyReLU (0.01),
 * the Extractor's 15-d sorted-key proprio features, a 3-d diagonal Gaussian
 * action head with state-independent log_std and a value head
 * (ballbot_rl/policies/mlp_policy.py:143-163, ballbot_rl/training/train.py:39-56);
 * per minibatch it does what PPO.train does between `for rollout_data in
 * get(batch_size)` and `optimizer.step()` (model.learn, train.py:284): the
 * forward pass, the loss of bb_ppo_loss, loss.backward(), clip_grad_norm_ and
 * AdamW.  The minibatch is perm[mb_counter][0..B) of the rollout arrays; the
 * loss terms go to log[row_counter][6] (loss, pg, vf, entropy loss, approx_kl,
 * clip_fraction); both counters are incremented on the device, so a captured
 * graph replays consecutive minibatches.  offsets: float offsets of the 21
 * parameter tensors in the flat buffer, each a multiple of 4, in the order
 * pi W0..W3, pi b0..b3, vf W0..W3, vf b0..b3, action W, action b, value W,
 * value b, log_std.  grad has the flat layout; entries outside the tensors are
 * never written (keep them 0).  B: a multiple of 256 in [256, 16384].
 * workspace: >= bb_ppo_mlp_workspace_bytes(B) bytes of device memory.
 * Five launches on stream; graph-capturable. */
typedef struct bb_ppo_mlp_args {
  float* params;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n_params;
  int32_t offsets[21];
  const float* obs;          /* [n][obs_dim] */
  const float* actions;      /* [n][3] unclipped */
  const float* old_logp;     /* [n] */
  const float* advantages;   /* [n] */
  const float* returns;      /* [n] */
  const int64_t* perm;       /* [n / B][B] */
  int64_t* mb_counter;
  int64_t* row_counter;
  float* log;
  const float* clip;         /* device scalars: clip range, learning rate */
  const float* lr;
  float* step;               /* AdamW step counter (float, as torch) */
  float* coef;               /* 4 floats of scratch */
  int32_t B;
  int32_t normalize_advantage;
  int32_t obs_dim;           /* 15 (proprio) or 56 (+ relative_image_timestamp, rgbd_0/1 features) */
  int32_t obs_direct;        /* 0: obs rows are perm-indexed rollout rows; 1: the minibatch's rows in order */
  float ent_coef, vf_coef;
  double beta1, beta2, eps, weight_decay, max_grad_norm;
  float* workspace;
  int64_t workspace_bytes;
  /* data-parallel update (ABI 18; update_mode="allreduce" over RCCL, ballbot_rl/training/ppo.py):
   * phase 0 runs the whole minibatch; phase 1 stops after the flat gradient (grad, the log row,
   * the counters); phase 2 runs only the clip + AdamW step over grad as it then is, its norm
   * taken from grad itself (after the caller's all-reduce of it).  adv_stats (device float[2]:
   * mean, 1 / (std + 1e-8)), when non-NULL, replaces the minibatch's own advantage
   * normalisation -- the global minibatch's statistics, from the ranks' all-reduce. */
  int32_t phase;
  const float* adv_stats;
} bb_ppo_mlp_args;
int bb_ppo_mlp_workspace_bytes(int B, int64_t* bytes);
int bb_ppo_mlp_step(const bb_ppo_mlp_args* args, void* stream);
/* The rollout's policy step for the same proprio MLP policy (SB3
 * ActorCriticPolicy.forward as called by OnPolicyAlgorithm.collect_rollouts,
 * model.learn at ballbot_rl/training/train.py:284): for n observation rows
 * obs_dev [n][obs_dim] (15, or 56 with the camera features), mean/value from the two trunks, actions = mean +
 * noise * exp(log_std) (noise_dev [n][3] standard normal; NULL = the mean),
 * their Gaussian log-probability and the value.  Writes actions_dev [n][3]
 * (unclipped, as SB3 stores them), values_dev [n], log_prob_dev [n], and
 * optionally clipped_dev [n][3] (clip to the [-1, 1] action space, what
 * env.step receives) and obs_copy_dev [n][15] (the rollout buffer's copy).
 * params_dev/offsets/n_params as for bb_ppo_mlp_step (every slot must lie inside
 * the n_params-float buffer).  One launch; graph-capturable. */
int bb_ppo_mlp_act(const float* params_dev, const int32_t* offsets, int64_t n_params, const float* obs_dev, int obs_dim,
                   const float* noise_dev, int n,
                   float* obs_copy_dev, float* actions_dev, float* clipped_dev, float* values_dev, float* log_prob_dev,
                   void* stream);
/* One whole PPO rollout of the proprio MLP policy in ONE launch (SB3
 * OnPolicyAlgorithm.collect_rollouts + Monitor, model.learn at
 * ballbot_rl/training/train.py:284): every env runs n_steps x (policy forward,
 * Gaussian sample a = mean + noise * exp(log_std), clip to [-1, 1], env.step,
 * bookkeeping) back to back -- the parameters are fixed during a rollout and the
 * envs are independent, so no step waits for the slowest env of the GPU.  The
 * policy (bb_ppo_mlp_act's, same params/offsets/n_params) runs fp32 on the env's
 * team, in another summation order than bb_ppo_mlp_act's MFMA tiles (equal to
 * fp32 rounding); the env step is bb_step_multi's (bit-identical to bb_step's
 * serial route for the same clipped actions).  Built-in rewards only (not
 * BB_REWARD_NONE).  One launch; graph-capturable.  On relief banks it runs as
 * bb_step_multi's relief pair (persistent, with the policy inside): a launch
 * that ends on the pair's wall-clock budget raises the handle's sticky fault
 * (bb_check), as bb_step_multi does. */
typedef struct bb_rollout_args {
  const float* params;      /* flat fp32 policy parameters, bb_ppo_mlp_act's slots, except that the eight
                               trunk weight matrices (slots 0-3, 8-11) are stored input-major (W^T,
                               [in][128]) so that a team's lanes read whole cache lines */
  int32_t offsets[21];
  int64_t n_params;
  const float* noise;       /* [T][n][3] standard normal draws */
  int n_steps;              /* T */
  float* obs;               /* [n][15] in: last observation; out: the observation after the rollout */
  uint8_t* last_starts;     /* [n] in/out: episode_starts */
  double* ep_ret;           /* [n] in/out: running episode return (float64, as Monitor) */
  int64_t* ep_len;          /* [n] in/out */
  float* buf_obs;           /* [T][n][15] */
  float* buf_actions;       /* [T][n][3] unclipped (as SB3 stores them) */
  float* buf_values;        /* [T][n] */
  float* buf_log_prob;      /* [T][n] */
  float* buf_rewards;       /* [T][n] */
  uint8_t* buf_starts;      /* [T][n] episode_starts of each step */
  double* ep_r_out;         /* [T][n] finished episodes' returns, NaN elsewhere */
  int64_t* ep_l_out;        /* [T][n] their lengths, 0 elsewhere */
} bb_rollout_args;
int bb_rollout(bb_handle* h, const bb_rollout_args* args, void* stream);
/* One rollout step's episode bookkeeping (SB3 collect_rollouts + Monitor,
 * model.learn at ballbot_rl/training/train.py:284): done = (flags_dev[i] &
 * done_mask) != 0; rewards_out_dev[i] = reward_dev[i]; the float64 episode
 * return ep_ret_dev and int64 length ep_len_dev accumulate, finished episodes
 * are written to ep_r_out_dev (NaN elsewhere) / ep_l_out_dev (0 elsewhere) and
 * their counters restart; starts_dev (and starts_next_dev unless NULL) get
 * done as uint8 (episode_starts of the next step).  One launch. */
int bb_rollout_track(const float* reward_dev, const uint8_t* flags_dev, int done_mask, int n, float* rewards_out_dev,
                     double* ep_ret_dev, int64_t* ep_len_dev, double* ep_r_out_dev, int64_t* ep_l_out_dev,
                     uint8_t* starts_dev, uint8_t* starts_next_dev, void* stream);
/* The camera policy's frozen depth encoder (the reference's rgbd branch with a
 * pretrained encoder: Conv2d(1,32,3,s2,p1) BatchNorm2d LeakyReLU, Conv2d(32,32,3,
 * s2,p1) BatchNorm2d LeakyReLU, Flatten, Linear(8192,20) BatchNorm1d Tanh;
 * ballbot_rl/encoders/models.py:6-54 as loaded by policies/mlp_policy.py:51-125)
 * over n 64x64 depth images (image i at images_dev + j * image_stride floats,
 * 16-byte aligned, with j = i, or j = index_dev[i] when index_dev is not NULL:
 * a minibatch read straight from the rollout buffer).  train != 0: the BatchNorms normalise with the batch's
 * statistics and update their running statistics and num_batches_tracked
 * (torch train mode, as SB3's policy.train() leaves them during PPO updates);
 * train == 0: the running statistics normalise (eval mode, the rollout).
 * Writes features row i at out_dev + i * out_stride (20 floats).  The pointers
 * in bb_encoder_params are the module's device tensors (running statistics and
 * counters are written in train mode; counters may be NULL).  Six launches on
 * stream; graph-capturable. */
typedef struct bb_encoder_params {
  const float *conv1_w, *conv1_b, *bn1_w, *bn1_b;
  float *bn1_mean, *bn1_var;
  int64_t* bn1_count;
  const float *conv2_w, *conv2_b, *bn2_w, *bn2_b;
  float *bn2_mean, *bn2_var;
  int64_t* bn2_count;
  const float *fc_w, *fc_b, *bn3_w, *bn3_b;
  float *bn3_mean, *bn3_var;
  int64_t* bn3_count;
} bb_encoder_params;
int bb_depth_encoder_workspace_bytes(int64_t n, int64_t* bytes);
int bb_depth_encoder(const bb_encoder_params* params, const float* images_dev, int64_t image_stride,
                     const int64_t* index_dev, int64_t n, int height, int width, int train, float momentum, float eps,
                     float* out_dev, int64_t out_stride, float* workspace_dev, int64_t workspace_bytes, void* stream);
/* copy terrain bank slot terrain_id (float32[293*293]) to host memory */
int bb_get_hfield(bb_handle* h, int terrain_id, float* data_host);
/* pin per-env terrain ids (device int32[n]) for every later reset; an id
 * outside [0, n_terrains) (e.g. -1) unpins the env (it draws from its stream
 * again).  A pinned reset takes no stream draw (a fixed config seed,
 * ballbot_env.py:505-510). */
int bb_assign_terrain(bb_handle* h, const int32_t* ids_dev, void* stream);
/* terrain seed streams as host tables (ballbot_env.py:378-384, 505-510): each reset of env e
 * that is not pinned takes the next draw of stream env_stream_host[e] (NULL:
 * all envs stream 0, n_streams must be 1): the k-th reset of the env (k = 0 at
 * the first reset after this call) gets bank slot slots_host[s * length + k],
 * i.e. the slot holding the terrain of the k-th value of the stream's
 * np_random(seed).integers(0, 10000).  Past `length` draws the stream wraps
 * around (counted in stats[5]).  Resets every env's draw counter to 0 and
 * turns off the device generators of bb_set_terrain_rng.  n_streams = 0
 * removes the streams (unpinned envs then reset onto slot 0).  Synchronous.
 * The table is refilled in place while n_streams * length fits the allocation
 * of an earlier call (a HIP graph captured before then reads the new table); a
 * larger table is a new allocation, and replaying a graph captured before that
 * call is invalid. */
int bb_set_terrain_stream(bb_handle* h, const int32_t* slots_host, int n_streams, int length,
                          const int32_t* env_stream_host);
/* terrain seed draws on the GPU, one numpy PCG64 generator per env
 * (gymnasium.utils.seeding.np_random = Generator(PCG64(SeedSequence(seed)))):
 * every reset of env e that is not pinned draws r_seed = integers(0, 10000)
 * from env e's generator (ballbot_env.py:505-510), bit-exact and without an
 * end, and resets onto bank slot seed_slot_host[r_seed] (seed_slot_host NULL:
 * slot == seed, the bank must hold all 10000 seeds; an entry of -1 marks a seed
 * that is not resident: such a draw is counted in stats[5] and takes slot
 * r_seed % n_terrains).  words_host uint64[n][5] is each generator's state as
 * numpy's PCG64.state holds it: state >> 64, state & (2^64-1), inc >> 64,
 * inc & (2^64-1), and (has_uint32 << 32) | uinteger.  words_host NULL turns
 * the device generators off.  Resets every env's draw counter to 0.
 * Synchronous; the buffers are allocated at the first call and refilled in
 * place, so a graph captured before a later call reads the new generators.
 * Replaces the per-env _np_random of BBotSimulation as SB3 seeds it: VecEnv.seed(seed)
 * then reset(seed=seed+i) (gymnasium Env.reset replaces _np_random,
 * ballbot_env.py:596; train.py:126-141), and an eval env's np_random(seed + N_ENVS + i)
 * (:378-384, train.py:90-97). */
int bb_set_terrain_rng(bb_handle* h, const uint64_t* words_host, const int32_t* seed_slot_host);
/* the device generators (uint64[n][5], as bb_set_terrain_rng takes them; may be
 * NULL) and the terrain seed of each env's last device draw (int32[n], -1 before
 * the first; may be NULL) */
int bb_get_terrain_rng(bb_handle* h, uint64_t* words_host, int32_t* last_seed_host);
/* current bank slot and number of stream draws of every env (host int32[n] each, may be NULL) */
int bb_get_env_terrain(bb_handle* h, int32_t* terrain_host, int32_t* draws_host);

/* reset envs where mask_dev[i] != 0 (mask NULL = all); writes reset obs.  A full reset (mask
 * NULL) clears the sticky fault of bb_check: when the fault is set it waits for `stream` so that
 * a bb_step* call straight after it steps (asynchronous, and capturable, otherwise). */
int bb_reset(bb_handle* h, const uint8_t* mask_dev, float* obs_dev, void* stream);

/* one env.step for all envs.  actions_dev float[n][3]; obs_dev float[n][15];
 * reward_dev float[n]; done_dev uint8[n]; terminal_obs_dev float[n][15] and
 * pos2d_dev float[n][2] may be NULL.  auto_reset != 0: done envs are reset in
 * the same launch and obs holds the reset observation (SB3 VecEnv). */
int bb_step(bb_handle* h, const float* actions_dev, float* obs_dev, float* reward_dev, uint8_t* done_dev,
            float* terminal_obs_dev, float* pos2d_dev, int auto_reset, void* stream);
/* k_steps consecutive env.steps of all envs in ONE launch, for action
 * sequences known in advance (open-loop: random-action benchmarks, replayed
 * actions): the same results as k_steps bb_step calls with actions_dev[k]
 * (bit-identical outputs, states, counters, auto-resets and terrain draws),
 * but each env runs its steps back to back instead of waiting at every step
 * for the slowest env on the GPU.  actions_dev float[k][n][3]; obs_dev
 * float[k][n][15]; reward_dev float[k][n]; done_dev uint8[k][n];
 * terminal_obs_dev float[k][n][15] and pos2d_dev float[k][n][2] may be NULL.
 * No reference counterpart (its VecEnv steps once per call,
 * ballbot_env.py:854); the per-step semantics are bb_step's.  On banks
 * without relief this is two launches on `stream`: the fast steps, with envs
 * whose step the fast path hands over parked at that step, then a finish
 * launch that resumes the parked envs (BB_MULTI_PARK=0 at bb_create: one
 * launch, hand-overs inline).  Relief banks: the relief pair -- one persistent
 * launch whose workgroups run either the fast or the full step, envs handed
 * between them through ticket rings per XCD label (BB_PAIR_ONE=0: two
 * concurrent launches; BB_RELIEF_PAIR=0: round 3's work queue) -- or, after a
 * launch in which no env needed a full step, the parked launches; a device flag
 * picks one per call (BB_MULTI_ADAPT=0: always the pair).  DESIGN §6d, §6e. */
int bb_step_multi(bb_handle* h, const float* actions_dev, int k_steps, float* obs_dev, float* reward_dev,
                  uint8_t* done_dev, float* terminal_obs_dev, float* pos2d_dev, int auto_reset, void* stream);

/* Wait for `stream` and report the handle's sticky fault: 0, or < 0 when a bb_step_multi
 * relief-pair launch ended on its wall-clock budget (BB_PAIR_BUDGET_MS, default 20 s: a team
 * waited that long for an env, which only a grid the device could not seat would cause).  The
 * launch then left some envs with their state at its start but terrain draws and counters
 * advanced, so from then on bb_step, bb_step_multi and bb_rollout return the same error at once
 * (no sync needed: the fault word is host memory mapped into the device) until a full bb_reset
 * (mask NULL) clears it.  No reference counterpart: MuJoCo's mj_step has no such launch. */
int bb_check(bb_handle* h, void* stream);

/* diagnostics / parity (synchronous, host arrays) */
int bb_get_state(bb_handle* h, double* qpos, double* qvel, double* warm, int32_t* steps);
int bb_set_state(bb_handle* h, const double* qpos, const double* qvel, const double* warm, const int32_t* steps);
int bb_forward(bb_handle* h, const double* ctrl, double* qacc, int32_t* ncontact);
/* the first n (<= BB_NSTATS) counters since create: [auto-resets, divergence resets (env-steps
 * with done bit 2), overflow (env-steps where a geom pair hit MuJoCo's mjMAXCONPAIR = 50 contacts and
 * was truncated, as MuJoCo does), slow-path env-steps (envs the fast kernel handed to the full
 * kernel: base-tree geom contacts possible), Newton iterations, resets past the end of their
 * terrain stream table or onto a drawn seed not resident in the bank, env-steps whose last RK stage stored base-tree contacts past the 32 LDS slots
 * (the per-env HBM spill block)] */
int bb_get_stats(bb_handle* h, int64_t* out, int n);
/* diagnostics of the last relief-pair launch of bb_step_multi (waits for the device): the first
 * n (<= BB_NPAIR) of [team-cycles stepping (fast, full), idle loop passes (fast, full), working
 * workgroups of the next launch (fast, full), env claims (fast, full), completed env-steps (fast,
 * full), fast-path hand-overs to the full launch, team lifetimes in shader cycles (fast, full), team
 * lifetimes in wall-clock ticks (fast, full), envs marked heavy for the solo waves, the ring length,
 * appends to the least-used fast ring and to the least-used full ring (laps = appends / length)].  No
 * reference counterpart (tools/). */
int bb_pair_counters(bb_handle* h, int64_t* out, int n);
/* per env, the last relief-pair launch (waits for the device): out[0:n] shader cycles its steps
 * took (its team's wave, lockstep included), out[n:2n] the wall-clock tick (bb_step_multi's
 * device wall clock) of its last step.  Diagnostics (tools/). */
int bb_pair_env_times(bb_handle* h, uint64_t* out);
/* launch configuration: [n_envs, envs_per_wave, fp64, lds_bytes_per_workgroup,
 * lanes_per_env] */
int bb_get_config(bb_handle* h, int32_t* out5);
/* init height offset per terrain (ballbot_env.py:546-563) */
int bb_get_offsets(bb_handle* h, float* out);
/* measurement: time the next max_launches fast step kernels (the dominant
 * kernel of bb_step) with HIP events on the caller's stream; bb_kernel_ms
 * waits for them and returns their average duration.  No reference
 * counterpart (bench.py's roofline.achieved). */
int bb_time_kernel(bb_handle* h, int max_launches);
int bb_kernel_ms(bb_handle* h, double* avg_ms, int32_t* launches);
/* the same timed steps, all three step kernels: avg_ms3 = [fast kernel, predicted full
 * kernel (route 0, concurrent on the handle's side stream; 0 when not launched),
 * hand-over full kernel (from the later of the two to its end)] */
int bb_kernel_times(bb_handle* h, double* avg_ms3, int32_t* launches);

#ifdef __cplusplus
}
#endif
#endif
