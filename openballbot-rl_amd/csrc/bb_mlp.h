// bb_mlp.h -- one fused PPO minibatch step of the reference's proprio MLP
// policy (bb_mlp.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

// Parameter slots in the flat fp32 buffer (float offsets, each a multiple of 4).
enum MlpSlot {
  MLP_PI_W0 = 0,  // pi trunk weights [128][15], [128][128] x3
  MLP_PI_B0 = 4,  // pi trunk biases [128] x4
  MLP_VF_W0 = 8,
  MLP_VF_B0 = 12,
  MLP_WA = 16,    // action_net [3][128]
  MLP_BA = 17,    // [3]
  MLP_WV = 18,    // value_net [1][128]
  MLP_BV = 19,    // [1]
  MLP_LS = 20,    // log_std [3]
  MLP_NSLOTS = 21
};

struct MlpStepArgs {
  float* params;        // flat fp32 parameters (AdamW updates them in place)
  float* grad;          // flat fp32 gradients, same layout (gaps stay 0)
  float* exp_avg;
  float* exp_avg_sq;
  long long n_params;   // flat length (with the alignment gaps)
  int off[MLP_NSLOTS];
  const float* obs;       // [n][in_dim] rollout observations (sorted-key proprio), or with
                          // obs_direct the minibatch's [B][in_dim] features in order
  int in_dim, obs_direct; // 15 (proprio) or 56 (+ relative_image_timestamp and the two camera features)
  const float* actions;   // [n][3] unclipped actions
  const float* old_logp;  // [n]
  const float* adv;       // [n]
  const float* returns;   // [n]
  const long long* perm;  // [nb][B] minibatch sample indices
  long long* mb_counter;  // minibatch within the epoch (read, then incremented)
  long long* row_counter; // log row (read, then incremented)
  float* log;             // [rows][6]: loss, pg, vf, ent, approx_kl, clip_fraction
  const float* clip;
  const float* lr;
  float* step;
  float* coef;            // [4] AdamW scratch
  int B, normalize;
  float ent_coef, vf_coef;
  double beta1, beta2, eps, weight_decay, max_norm;
  float* ws;
  long long ws_bytes;
  // data-parallel update: phase 0 the whole minibatch, 1 up to the flat gradient (no optimiser
  // step), 2 clip + AdamW over the gradient as it then is (after the ranks' all-reduce);
  // adv_stats (device [2]: mean, 1 / (std + 1e-8)) replaces the minibatch's own advantage
  // normalisation (the global minibatch's statistics), NULL: the minibatch's own
  int phase = 0;
  const float* adv_stats = nullptr;
};

// the rollout's policy step (SB3 ActorCriticPolicy.forward) for n obs rows
struct MlpActArgs {
  const float* params;
  int off[MLP_NSLOTS];
  const float* obs;      // [n][in_dim]
  int in_dim;            // 15 or 56
  const float* noise;    // [n][3] or NULL (deterministic)
  int n;
  float* obs_copy;       // [n][in_dim] or NULL
  float* actions;        // [n][3] unclipped
  float* clipped;        // [n][3] or NULL
  float* values;         // [n]
  float* log_prob;       // [n]
};

long long mlp_workspace_bytes(int B);
int launch_mlp_act(const MlpActArgs& a, hipStream_t s);
int launch_mlp_step(const MlpStepArgs& a, hipStream_t s);

}  // namespace bb
