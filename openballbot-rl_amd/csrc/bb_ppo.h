// bb_ppo.h -- fused PPO minibatch loss (bb_ppo.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

struct PPOLossArgs {
  const float* mean;      // [B][3] policy means
  const float* values;    // [B]
  const float* log_std;   // [3]
  const float* actions;   // [B][3] stored (unclipped) actions
  const float* old_logp;  // [B]
  const float* adv;       // [B]
  const float* returns;   // [B]
  const float* clip;      // device scalar (graph-replayable)
  int B, normalize;
  float ent_coef, vf_coef;
  float* terms;           // [9]: loss, pg, vf, ent, approx_kl, clip_fraction, dloss/dls[3]
  float* grad_mean;       // [B][3]
  float* grad_values;     // [B]
};

int launch_ppo_loss(const PPOLossArgs& a, hipStream_t s);

}  // namespace bb
