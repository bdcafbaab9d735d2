// bb_rollout.h -- rollout-buffer kernels (bb_rollout.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

// GAE over [T][N] float32 rollouts (SB3 RolloutBuffer.compute_returns_and_advantage)
int launch_gae(const float* rew, const float* val, const uint8_t* start, const float* last_val,
               const uint8_t* last_done, int T, int N, double gamma, double lam, float* adv, float* ret,
               hipStream_t s);

}  // namespace bb
