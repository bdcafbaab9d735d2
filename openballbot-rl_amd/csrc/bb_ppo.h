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

// clip_grad_norm_ + AdamW on flat fp32 buffers (bb_adamw_clip)
struct AdamWArgs {
  float* param;            // [n]
  const float* grad;       // [n] (not modified; the clip factor is applied on the fly)
  float* exp_avg;          // [n]
  float* exp_avg_sq;       // [n]
  long long n;
  const float* lr;         // device scalar (graph-replayable schedule)
  float* step;             // device scalar, incremented once per call (torch's float32 step)
  float* coef;             // device scratch [4]: clip factor, step size, sqrt(1 - b2^t), 1 - lr wd
  // torch takes the hyper-parameters as Python doubles: 1 - beta etc. are
  // formed in double and rounded once, as its kernels receive them
  double beta1, beta2;     // bias corrections beta^t (double, as torch's eager AdamW)
  double weight_decay;
  float b2, omb1, omb2;    // float(beta2), float(1 - beta1), float(1 - beta2)
  float eps, max_norm;
  // optional: per-workgroup partial sums of g^2 (bb_mlp.hip writes them while
  // it assembles the gradient); NULL = the prep launch reduces grad itself
  const float* norm_part;
  int n_norm_part;
};

int launch_adamw_clip(const AdamWArgs& a, hipStream_t s);

}  // namespace bb
