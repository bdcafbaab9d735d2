// bb_rollout.h -- rollout-buffer kernels (bb_rollout.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

// GAE over [T][N] float32 rollouts (SB3 RolloutBuffer.compute_returns_and_advantage)
int launch_gae(const float* rew, const float* val, const uint8_t* start, const float* last_val,
               const uint8_t* last_done, int T, int N, double gamma, double lam, float* adv, float* ret,
               hipStream_t s);

// one rollout step's episode bookkeeping (SB3 collect_rollouts + Monitor)
int launch_track(const float* reward, const uint8_t* flags, int mask, int n, float* rewards_out, double* ep_ret,
                 long long* ep_len, double* ep_r_out, long long* ep_l_out, uint8_t* starts, uint8_t* starts_next,
                 hipStream_t s);

}  // namespace bb
