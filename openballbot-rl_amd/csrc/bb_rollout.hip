// bb_rollout.hip -- rollout-buffer kernels of the PPO update boundary.
//
// GAE(gamma, lambda) over a [T][N] rollout, one thread per env walking time
// backwards: the restatement of stable-baselines3 2.6.0
// RolloutBuffer.compute_returns_and_advantage (the reference trains with SB3
// PPO, ballbot_rl/training/train.py:125-142).  SB3 evaluates it in numpy
// float32 with Python-float coefficients, i.e. f32(gamma) and f32(gamma*lambda):
//   delta_t = r_t + g * V_{t+1} * nnt_{t+1} - V_t
//   A_t     = delta_t + gl * nnt_{t+1} * A_{t+1}
//   R_t     = A_t + V_t
// with nnt_{t+1} = 1 - episode_start_{t+1} (t < T-1) or 1 - last_done, and
// V_T = last_value.  Contraction is off, so the result is bit-identical to
// that float32 sequence (tests/test_gpu_ppo.py).
//
// HBM bound: per env-step reads r, V (4 B each) and the start flag (1 B) and
// writes A, R (4 B each) -- 17 B; a [T][N] layout makes every time slice one
// coalesced row of N.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_rollout.h"

namespace bb {
namespace {

__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const uint8_t* __restrict__ start, const float* __restrict__ last_val,
                                                  const uint8_t* __restrict__ last_done, int T, int N, float g,
                                                  float gl, float* __restrict__ adv, float* __restrict__ ret) {
#pragma clang fp contract(off)
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  float next_v = last_val[e];
  float nnt = 1.0f - float(last_done[e] != 0);
  float a = 0.0f;
  for (int t = T - 1; t >= 0; t--) {
    const size_t i = size_t(t) * N + e;
    const float v = val[i];
    const float delta = rew[i] + g * next_v * nnt - v;
    a = delta + gl * nnt * a;
    adv[i] = a;
    ret[i] = a + v;
    next_v = v;
    nnt = 1.0f - float(start[i] != 0);
  }
}

// Episode bookkeeping of one rollout step (SB3 OnPolicyAlgorithm.collect_rollouts
// + Monitor): store the reward, accumulate the per-env return (float64, as
// Monitor sums Python floats) and length, record finished episodes (return,
// length; NaN / 0 elsewhere) and restart the counters, and publish
// episode_starts for the next step.  done = (flags & mask) != 0.
__global__ __launch_bounds__(256) void track_kernel(const float* __restrict__ reward, const uint8_t* __restrict__ flags,
                                                    int mask, int n, float* __restrict__ rewards_out,
                                                    double* __restrict__ ep_ret, long long* __restrict__ ep_len,
                                                    double* __restrict__ ep_r_out, long long* __restrict__ ep_l_out,
                                                    uint8_t* __restrict__ starts, uint8_t* __restrict__ starts_next) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float r = reward[e];
  const bool done = (flags[e] & mask) != 0;
  rewards_out[e] = r;
  const double ret = ep_ret[e] + double(r);
  const long long len = ep_len[e] + 1;
  ep_r_out[e] = done ? ret : __builtin_nan("");
  ep_l_out[e] = done ? len : 0;
  ep_ret[e] = done ? 0.0 : ret;
  ep_len[e] = done ? 0 : len;
  starts[e] = done ? 1 : 0;
  if (starts_next) starts_next[e] = done ? 1 : 0;
}

}  // namespace

int launch_track(const float* reward, const uint8_t* flags, int mask, int n, float* rewards_out, double* ep_ret,
                 long long* ep_len, double* ep_r_out, long long* ep_l_out, uint8_t* starts, uint8_t* starts_next,
                 hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(track_kernel, dim3((n + 255) / 256), dim3(256), 0, s, reward, flags, mask, n, rewards_out, ep_ret,
                     ep_len, ep_r_out, ep_l_out, starts, starts_next);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gae(const float* rew, const float* val, const uint8_t* start, const float* last_val,
               const uint8_t* last_done, int T, int N, double gamma, double lam, float* adv, float* ret,
               hipStream_t s) {
  if (T <= 0 || N <= 0) return 0;
  hipLaunchKernelGGL(gae_kernel, dim3((N + 255) / 256), dim3(256), 0, s, rew, val, start, last_val, last_done, T, N,
                     float(gamma), float(gamma * lam), adv, ret);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
