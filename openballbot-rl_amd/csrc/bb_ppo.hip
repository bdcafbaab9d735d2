// bb_ppo.hip -- fused PPO minibatch loss + gradients.
//
// SB3 2.6.0 PPO.train evaluates, per minibatch of B samples (the reference's
// PPO, ballbot_rl/training/train.py:125-142), with a diagonal Gaussian policy:
//   lp_i   = sum_j -z_ij^2/2 - ls_j - log(2 pi)/2,  z_ij = (a_ij - mu_ij) e^-ls_j
//   rho_i  = exp(lp_i - old_lp_i)
//   A_i    = adv_i, or (adv_i - mean) / (std + 1e-8) when normalize_advantage
//   pg     = -mean_i min(A_i rho_i, A_i clip(rho_i, 1-c, 1+c))
//   vf     = mean_i (R_i - V_i)^2
//   ent    = -mean_i sum_j (1/2 + log(2 pi)/2 + ls_j)
//   loss   = pg + ent_coef ent + vf_coef vf
//   kl     = mean_i (rho_i - 1) - (lp_i - old_lp_i);  clip_fraction = mean_i [|rho_i - 1| > c]
// Eager PyTorch spends ~50 small kernels on this; here it is one launch that
// also writes d loss / d(mu, V, ls) for the backward pass.  The min() gradient
// follows torch.minimum (ties split evenly, so rho inside the clip range gets
// the full -A), clamp passes gradient inside [1-c, 1+c].
//
// One 1024-thread workgroup: B = 8192 is 8 samples per thread; the sums are
// wave shuffles + one LDS pass.  Traffic per sample: 9 floats in, 4 out.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_ppo.h"

namespace bb {
namespace {

constexpr int PPO_THREADS = 1024;
constexpr int NACC = 8;  // pg, vf, kl, cf, dls0..2, (pad)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// block-wide sums of NACC values; every thread gets the totals
__device__ void block_sums(float (&v)[NACC], float (*red)[NACC]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NACC; k++) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NACC; k++) red[wid][k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NACC; k++) {
    float s = 0.f;
    for (int w = 0; w < PPO_THREADS / 64; w++) s += red[w][k];
    v[k] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(PPO_THREADS) void ppo_loss_kernel(PPOLossArgs p) {
  __shared__ float red[PPO_THREADS / 64][NACC];
  const float c = *p.clip;
  const float ls[3] = {p.log_std[0], p.log_std[1], p.log_std[2]};
  const float inv_std[3] = {expf(-ls[0]), expf(-ls[1]), expf(-ls[2])};
  const float half_log_2pi = 0.91893853320467274f;
  const float lp_const = -(ls[0] + ls[1] + ls[2]) - 3.f * half_log_2pi;
  const int B = p.B;
  const float invB = 1.f / float(B);
  // advantage normalisation (torch.std: unbiased)
  float amean = 0.f, ainv = 1.f;
  if (p.normalize && B > 1) {
    float v[NACC] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < B; i += PPO_THREADS) { const float a = p.adv[i]; v[0] += a; }
    block_sums(v, red);
    amean = v[0] * invB;
    float w[NACC] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < B; i += PPO_THREADS) { const float d = p.adv[i] - amean; w[0] += d * d; }
    block_sums(w, red);
    ainv = 1.f / (sqrtf(w[0] / float(B - 1)) + 1e-8f);
  }
  float acc[NACC] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = threadIdx.x; i < B; i += PPO_THREADS) {
    float z[3], lp = lp_const;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      z[j] = (p.actions[3 * i + j] - p.mean[3 * i + j]) * inv_std[j];
      lp -= 0.5f * z[j] * z[j];
    }
    const float lr = lp - p.old_logp[i];
    const float rho = expf(lr);
    const float A = p.normalize && B > 1 ? (p.adv[i] - amean) * ainv : p.adv[i];
    const float rc = fminf(fmaxf(rho, 1.f - c), 1.f + c);
    const float s1 = A * rho, s2 = A * rc;
    acc[0] += -fminf(s1, s2);
    const float e = p.returns[i] - p.values[i];
    acc[1] += e * e;
    acc[2] += (rho - 1.f) - lr;
    acc[3] += fabsf(rho - 1.f) > c ? 1.f : 0.f;
    // d pg_i / d rho: -A through the unclipped branch, or the clipped one inside the range
    const bool inside = rho >= 1.f - c && rho <= 1.f + c;
    const float gr = (inside || s1 < s2) ? -A : 0.f;
    const float glp = gr * rho * invB;  // d loss / d lp_i
#pragma unroll
    for (int j = 0; j < 3; j++) {
      p.grad_mean[3 * i + j] = glp * z[j] * inv_std[j];
      acc[4 + j] += glp * (z[j] * z[j] - 1.f);
    }
    p.grad_values[i] = p.vf_coef * 2.f * (p.values[i] - p.returns[i]) * invB;
  }
  block_sums(acc, red);
  if (threadIdx.x == 0) {
    const float pg = acc[0] * invB, vf = acc[1] * invB;
    const float ent = -(3.f * (0.5f + half_log_2pi) + ls[0] + ls[1] + ls[2]);
    p.terms[0] = pg + p.ent_coef * ent + p.vf_coef * vf;
    p.terms[1] = pg;
    p.terms[2] = vf;
    p.terms[3] = ent;
    p.terms[4] = acc[2] * invB;
    p.terms[5] = acc[3] * invB;
#pragma unroll
    for (int j = 0; j < 3; j++) p.terms[6 + j] = acc[4 + j] - p.ent_coef;  // d loss / d ls_j
  }
}

}  // namespace

int launch_ppo_loss(const PPOLossArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  hipLaunchKernelGGL(ppo_loss_kernel, dim3(1), dim3(PPO_THREADS), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
