// bb_mlp.hip -- one PPO minibatch of the reference's proprio policy, fused
// (SURVEY.md §8 F1): forward of both 4x128 LeakyReLU trunks, the Gaussian and
// value heads, SB3 2.6.0's PPO loss and its gradients, the backward pass, the
// weight gradients, clip_grad_norm_ and AdamW -- five launches instead of the
// ~50 PyTorch/hipBLASLt launches of the autograd path.
//
// The policy (ballbot_rl/policies/mlp_policy.py:143-163, train.py:39-56):
//   f = obs: 15 sorted-key proprio floats, or the camera policy's 56 features
//       (proprio, relative_image_timestamp, the two frozen-encoder outputs)
//   pi: h1..h4 = leaky(h W^T + b), IN->128->128->128->128;  mean = h4 Wa^T + ba (3)
//   vf: the same trunk shape;                               value = h4 Wv^T + bv (1)
// The loss is bb_ppo.hip's (clipped surrogate, MSE value loss, entropy of a
// state-independent log_std); its per-sample gradient needs only the
// minibatch's advantage mean/std, which every tile recomputes (same order, so
// the same bits), so the gradient flows back through the tile that formed it.
//
// Launches (B = minibatch rows, tiles of 32 rows):
//   1. mlp_tile_kernel<TRAIN, IN>  B/32 workgroups x 8 waves: waves 0-3 the pi
//      trunk, 4-7 the vf trunk; wave w owns columns 32(w%4)..+31 of every
//      128-wide layer.  A 128->128 layer is 64 v_mfma_f32_32x32x2_f32 per wave
//      with the layer input read from an LDS tile (float4 per lane, k order
//      permuted identically for A and B) and W from L2; the input layer takes
//      (IN+1)/2 steps.  Activations stay in registers in the MFMA C layout for
//      the LeakyReLU backward; the heads and the loss run on the VALU.
//      Backward: dh_l = dz_{l+1} W_l (MFMA again).  Layer inputs h_l and output
//      gradients dz_{l+1} go to a workspace for launch 2; loss terms leave as
//      per-tile partials.  TRAIN = false is the rollout's policy step.
//   2. mlp_dw_kernel     dW_l = dz_{l+1}^T h_l and db_l = dz_{l+1}^T 1 over
//      row chunks: one workgroup per (layer, chunk) stages 32-row slabs of dz
//      and h in LDS; wave w owns output rows 32w..32w+31, all columns.
//   3. mlp_reduce_kernel sums the chunk partials in a fixed order into the
//      flat gradient buffer, g^2 per workgroup for the clip, the log_std
//      gradient, the log row, and advances the minibatch/log-row counters
//      (graph replays).
//   4-5. bb_ppo.hip's adamw_prep/adamw_update (clip factor from the partials).
// fp32 throughout (the MFMA is exact f32); only summation orders differ from
// autograd (tests/test_gpu_ppo.py: test_fused_minibatch_matches_autograd).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_mlp.h"
#include "bb_ppo.h"

namespace bb {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int HID = 128;          // trunk width
constexpr int IN_MAX = 56;        // policy input features: 15 (proprio) or 56 (with the camera features)
constexpr int XW_MAX = 64;        // workspace row width of the padded input
constexpr int ROWS = 32;          // rows per tile (the MFMA M)
constexpr int T1 = 512;           // threads per tile workgroup: 8 waves = 2 trunks x 4 column blocks
constexpr int LDT = HID + 4;      // LDS row stride (floats): float4 rows, no bank conflicts
constexpr int MAXCH = 64;         // max K chunks of the weight-gradient GEMMs
constexpr int LPART = 8;          // loss partials per tile: pg, vf, kl, cf, dls[3], -
constexpr int NJOB = 10;          // weight-gradient GEMMs: 2 trunks x 4 layers + 2 heads
constexpr int NSEG = 2 * NJOB;    // gradient segments: weights and biases of each job
constexpr int SLAB = 32;          // rows per LDS slab in the dW kernel
constexpr float SLOPE = 0.01f;    // nn.LeakyReLU default negative_slope
constexpr float HALF_LOG_2PI = 0.91893853320467274f;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// C/D layout of the 32x32 f32 MFMA: column = lane & 31, row = crow(reg, lane)
__device__ __forceinline__ int crow(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ float leaky(float z) { return z > 0.f ? z : z * SLOPE; }

// K chunks of the weight-gradient GEMMs: the most (<= MAXCH) whose chunk is a
// whole number of SLAB-row slabs
__host__ __device__ inline int n_chunks(int B) {
  for (int c = MAXCH; c > 1; c >>= 1)
    if (B % (c * SLAB) == 0) return c;
  return 1;
}
constexpr int WELEMS = 2 * (HID * IN_MAX + 3 * HID * HID) + 4 * HID;  // weight elements (upper bound)
constexpr int BELEMS = 2 * 4 * HID + 4;                           // bias elements

struct Workspace {
  float* x;           // [B][32] padded inputs
  float* h[2][4];     // [B][128] h1..h4 per trunk
  float* dz[2][4];    // [B][128] dL/dz of layers 0..3 per trunk
  float* dhead;       // [B][4] dL/dmean[3], dL/dvalue
  float* lpart;       // [B/32][LPART]
  float* wpart;       // [nch][weights] per job
  float* bpart;       // [nch][biases] per job
  float* npart;       // [reduce workgroups]
};

Workspace carve(float* base, int B, long long* total_floats) {
  Workspace w;
  long long o = 0;
  auto take = [&](long long n) { float* p = base ? base + o : nullptr; o += (n + 63) & ~63LL; return p; };
  w.x = take((long long)B * XW_MAX);
  for (int t = 0; t < 2; t++)
    for (int l = 0; l < 4; l++) w.h[t][l] = take((long long)B * HID);
  for (int t = 0; t < 2; t++)
    for (int l = 0; l < 4; l++) w.dz[t][l] = take((long long)B * HID);
  w.dhead = take((long long)B * 4);
  w.lpart = take((long long)(B / ROWS) * LPART);
  w.wpart = take((long long)MAXCH * WELEMS);
  w.bpart = take((long long)MAXCH * BELEMS);
  w.npart = take(4096);
  if (total_floats) *total_floats = o;
  return w;
}

struct TileArgs {
  const float* P;
  int off[MLP_NSLOTS];
  const float* obs;
  const float* actions;
  const float* old_logp;
  const float* adv;
  const float* returns;
  const long long* perm;
  const long long* mb_counter;
  const float* clip;
  const float* adv_stats;  // TRAIN: external advantage normalisation [mean, 1/(std+1e-8)], or NULL
  int B, normalize;
  float vf_coef;
  Workspace w;
  int obs_direct;  // TRAIN: obs rows are the minibatch in order (not indexed by perm)
  // rollout (act) mode: rows r0.. of obs directly, n of them
  int n;
  const float* noise;   // [n][3] standard normal draws, NULL = deterministic (the mean)
  float* obs_copy;      // [n][15] or NULL
  float* act_out;       // [n][3] unclipped actions
  float* act_clipped;   // [n][3] actions clipped to [-1, 1] or NULL
  float* values_out;    // [n]
  float* logp_out;      // [n]
};

// block-wide sum over the T1 threads, same order in every workgroup
__device__ float block_sum(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
}

// store a wave's 32x32 C-layout block: rows of the tile, column col
__device__ __forceinline__ void store_block(const f32x16& v, float* dst, int ld, int col, int lane) {
#pragma unroll
  for (int r = 0; r < 16; r++) dst[(long long)crow(r, lane) * ld + col] = v[r];
}

// one 128->128 product of a 32-row tile for this wave's 32 output columns:
// acc += A (LDS tile, rows x K) * B, B[k][col] = wk(k) -- forward: W[col][k]
// (float4 along k), backward: W[k][col]
template <bool FWD>
__device__ __forceinline__ f32x16 tile_gemm(f32x16 acc, const float* tile_row, const float* W, int col, int hh) {
  // every W operand of the layer is requested before the first MFMA (64 VGPRs),
  // so the L2 latency is paid once per layer, not once per unrolled group
  const float* arow = tile_row + 4 * hh;
  float4 b4[HID / 8];
  if (FWD) {
    const float* wrow = W + col * HID + 4 * hh;
#pragma unroll
    for (int m = 0; m < HID / 8; m++) b4[m] = *reinterpret_cast<const float4*>(wrow + 8 * m);
  } else {
    const float* wcol = W + 4 * hh * HID + col;
#pragma unroll
    for (int m = 0; m < HID / 8; m++) {
      const float* wp = wcol + 8 * m * HID;
      b4[m] = make_float4(wp[0], wp[HID], wp[2 * HID], wp[3 * HID]);
    }
  }
#pragma unroll
  for (int m = 0; m < HID / 8; m++) {
    const float4 a4 = *reinterpret_cast<const float4*>(arow + 8 * m);
    acc = mfma(a4.x, b4[m].x, acc);
    acc = mfma(a4.y, b4[m].y, acc);
    acc = mfma(a4.z, b4[m].z, acc);
    acc = mfma(a4.w, b4[m].w, acc);
  }
  return acc;
}

// TRAIN: one minibatch tile of the update (forward, loss, backward).
// !TRAIN: the rollout's policy step, SB3 ActorCriticPolicy.forward over obs rows.
// IN: policy input features (15 proprio, 56 with the camera features); the
// padded input is XW wide in the workspace.
template <bool TRAIN, int IN>
__global__ __launch_bounds__(T1) void mlp_tile_kernel(TileArgs p) {
  constexpr int XW = IN <= 16 ? 32 : 64;
  constexpr int LDX = IN + 2;
  __shared__ __attribute__((aligned(16))) float xs[2][2][ROWS][LDT];  // [trunk][buffer] exchange tiles
  __shared__ float xin[ROWS][LDX];
  __shared__ float head[ROWS][4];  // dL/dmean[3], dL/dvalue
  __shared__ float hm[ROWS][4];    // mean[3], value
  __shared__ float red[8];
  __shared__ int idx[ROWS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5;
  const int t = w >> 2;                           // trunk: 0 pi, 1 vf
  const int col = (w & 3) * 32 + (lane & 31);     // this lane's output column
  const int B = p.B, tile = blockIdx.x, r0 = tile * ROWS;
  const long long* perm = TRAIN ? p.perm + (*p.mb_counter) * (long long)B : nullptr;
  const float* P = p.P;

  // advantage normalisation over the minibatch (torch.std: unbiased), one pass
  // over memory: each thread keeps its samples in registers
  float amean = 0.f, ainv = 1.f;
  if (TRAIN && p.normalize && B > 1 && p.adv_stats) {  // the global minibatch's (data-parallel update)
    amean = p.adv_stats[0];
    ainv = p.adv_stats[1];
  } else if (TRAIN && p.normalize && B > 1) {
    constexpr int MAXPT = 32;  // B <= 16384 keeps every sample in registers
    float v[MAXPT];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXPT; j++) {
      const int i = tid + j * T1;
      v[j] = i < B ? p.adv[perm[i]] : 0.f;
      s += v[j];
    }
    for (int i = tid + MAXPT * T1; i < B; i += T1) s += p.adv[perm[i]];
    amean = block_sum(s, red) / float(B);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < MAXPT; j++) {
      const float d = v[j] - amean;
      q += tid + j * T1 < B ? d * d : 0.f;
    }
    for (int i = tid + MAXPT * T1; i < B; i += T1) { const float d = p.adv[perm[i]] - amean; q += d * d; }
    ainv = 1.f / (sqrtf(block_sum(q, red) / float(B - 1)) + 1e-8f);
  }

  if (tid < ROWS) idx[tid] = TRAIN ? (int)perm[r0 + tid] : (r0 + tid < p.n ? r0 + tid : -1);
  __syncthreads();
  for (int e = tid; e < ROWS * XW; e += T1) {
    const int r = e / XW, c = e % XW, i = idx[r];
    // obs_direct: the input rows are already the minibatch, in order (camera features)
    const long long src = TRAIN && p.obs_direct ? (long long)(r0 + r) : (long long)i;
    const float v = c < IN && i >= 0 ? p.obs[src * IN + c] : 0.f;
    if (c < LDX) xin[r][c] = v;
    if (TRAIN) p.w.x[(long long)(r0 + r) * XW + c] = v;
    if (!TRAIN && p.obs_copy && c < IN && i >= 0) p.obs_copy[(long long)i * IN + c] = v;
  }
  __syncthreads();

  // ---------------- forward: waves 0-3 the pi trunk, 4-7 the vf trunk, in lockstep
  const int wbase = t ? MLP_VF_W0 : MLP_PI_W0, bbase = t ? MLP_VF_B0 : MLP_PI_B0;
  f32x16 hreg[4];
  int cur = 0;
  {  // layer 0, K = IN (padded to even)
    f32x16 acc;
    const float bias = P[p.off[bbase] + col];
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = bias;
    const float* W0 = P + p.off[wbase] + col * IN;
#pragma unroll
    for (int s = 0; s < (IN + 1) / 2; s++) {
      const int k = 2 * s + hh;
      acc = mfma(k < IN ? xin[lane & 31][k] : 0.f, k < IN ? W0[k] : 0.f, acc);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = leaky(acc[r]);
    hreg[0] = acc;
    if (TRAIN) store_block(acc, p.w.h[t][0] + (long long)r0 * HID, HID, col, lane);
    store_block(acc, &xs[t][cur][0][0], LDT, col, lane);
    __syncthreads();
  }
#pragma unroll
  for (int l = 1; l < 4; l++) {
    f32x16 acc;
    const float bias = P[p.off[bbase + l] + col];
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = bias;
    acc = tile_gemm<true>(acc, &xs[t][cur][lane & 31][0], P + p.off[wbase + l], col, hh);
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = leaky(acc[r]);
    hreg[l] = acc;
    if (TRAIN) store_block(acc, p.w.h[t][l] + (long long)r0 * HID, HID, col, lane);
    store_block(acc, &xs[t][cur ^ 1][0][0], LDT, col, lane);
    cur ^= 1;
    __syncthreads();
  }
  // heads on h4 (xs[t][cur]): threads of trunk t, (row, 16-column part)
  {
    const int tt = tid >> 8, r = (tid >> 3) & 31, part = tid & 7;
    const float* hrow = &xs[tt][cur][r][part * 16];
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    if (tt == 0) {
      const float* Wa = P + p.off[MLP_WA] + part * 16;
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const float h = hrow[c];
        s0 += h * Wa[c];
        s1 += h * Wa[HID + c];
        s2 += h * Wa[2 * HID + c];
      }
    } else {
      const float* Wv = P + p.off[MLP_WV] + part * 16;
#pragma unroll
      for (int c = 0; c < 16; c++) s0 += hrow[c] * Wv[c];
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      s0 += __shfl_xor(s0, off, 64);
      s1 += __shfl_xor(s1, off, 64);
      s2 += __shfl_xor(s2, off, 64);
    }
    if (part == 0) {
      if (tt == 0) {
        hm[r][0] = s0 + P[p.off[MLP_BA]];
        hm[r][1] = s1 + P[p.off[MLP_BA] + 1];
        hm[r][2] = s2 + P[p.off[MLP_BA] + 2];
      } else {
        hm[r][3] = s0 + P[p.off[MLP_BV]];
      }
    }
  }
  __syncthreads();

  if (!TRAIN) {  // SB3 DiagGaussian: a = mean + eps * exp(log_std); log_prob of a; value
    if (w != 0 || lane >= ROWS || idx[lane] < 0) return;
    const int r = lane, i = idx[r];
    const float* ls = P + p.off[MLP_LS];
    float lp = 0.f;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const float mu = hm[r][j];
      const float a = p.noise ? __fadd_rn(mu, __fmul_rn(p.noise[3LL * i + j], expf(ls[j]))) : mu;
      const float z = __fmul_rn(__fsub_rn(a, mu), expf(-ls[j]));
      lp += -0.5f * z * z - ls[j] - 0.5f * (2.f * HALF_LOG_2PI);
      p.act_out[3LL * i + j] = a;
      if (p.act_clipped) p.act_clipped[3LL * i + j] = fminf(fmaxf(a, -1.f), 1.f);
    }
    p.values_out[i] = hm[r][3];
    p.logp_out[i] = lp;
    return;
  }

  // ---------------- loss (SB3 PPO.train, bb_ppo.hip) and head gradients: wave 0, lane = row
  if (w == 0) {
    const float c = *p.clip;
    const float* ls = P + p.off[MLP_LS];
    const float l0 = ls[0], l1 = ls[1], l2 = ls[2];
    const float inv_std[3] = {expf(-l0), expf(-l1), expf(-l2)};
    const float lp_const = -(l0 + l1 + l2) - 3.f * HALF_LOG_2PI;
    const float invB = 1.f / float(B);
    float acc[7] = {0, 0, 0, 0, 0, 0, 0};
    if (lane < ROWS) {
      const int r = lane, i = idx[r];
      float z[3], lp = lp_const;
#pragma unroll
      for (int j = 0; j < 3; j++) {
        z[j] = (p.actions[3LL * i + j] - hm[r][j]) * inv_std[j];
        lp -= 0.5f * z[j] * z[j];
      }
      const float lr = lp - p.old_logp[i];
      const float rho = expf(lr);
      const float A = p.normalize && B > 1 ? (p.adv[i] - amean) * ainv : p.adv[i];
      const float rc = fminf(fmaxf(rho, 1.f - c), 1.f + c);
      const float s1 = A * rho, s2 = A * rc;
      acc[0] = -fminf(s1, s2);
      const float e = p.returns[i] - hm[r][3];
      acc[1] = e * e;
      acc[2] = (rho - 1.f) - lr;
      acc[3] = fabsf(rho - 1.f) > c ? 1.f : 0.f;
      const bool inside = rho >= 1.f - c && rho <= 1.f + c;
      const float gr = (inside || s1 < s2) ? -A : 0.f;
      const float glp = gr * rho * invB;
      float gh[4];
#pragma unroll
      for (int j = 0; j < 3; j++) {
        gh[j] = glp * z[j] * inv_std[j];
        acc[4 + j] = glp * (z[j] * z[j] - 1.f);
      }
      gh[3] = p.vf_coef * 2.f * (hm[r][3] - p.returns[i]) * invB;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        head[r][j] = gh[j];
        p.w.dhead[(long long)(r0 + r) * 4 + j] = gh[j];
      }
    }
    // tile sums over the 32 rows (lanes 32..63 hold zeros)
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
      for (int q = 0; q < 7; q++) acc[q] += __shfl_xor(acc[q], off, 64);
    }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 7; q++) p.w.lpart[(long long)tile * LPART + q] = acc[q];
      p.w.lpart[(long long)tile * LPART + 7] = 0.f;
    }
  }
  __syncthreads();

  // ---------------- backward, both trunks in lockstep
  f32x16 dz;
  {
    const float* Wh = P + p.off[t ? MLP_WV : MLP_WA];
    const float w0 = Wh[col];
    const float w1 = t ? 0.f : Wh[HID + col];
    const float w2 = t ? 0.f : Wh[2 * HID + col];
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int R = crow(r, lane);
      const float d = t ? head[R][3] * w0 : (head[R][0] * w0 + head[R][1] * w1) + head[R][2] * w2;
      dz[r] = hreg[3][r] > 0.f ? d : d * SLOPE;
    }
  }
#pragma unroll
  for (int l = 3; l >= 1; l--) {
    store_block(dz, p.w.dz[t][l] + (long long)r0 * HID, HID, col, lane);
    store_block(dz, &xs[t][cur][0][0], LDT, col, lane);
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = 0.f;
    acc = tile_gemm<false>(acc, &xs[t][cur][lane & 31][0], P + p.off[wbase + l], col, hh);
#pragma unroll
    for (int r = 0; r < 16; r++) dz[r] = hreg[l - 1][r] > 0.f ? acc[r] : acc[r] * SLOPE;
    cur ^= 1;
  }
  store_block(dz, p.w.dz[t][0] + (long long)r0 * HID, HID, col, lane);
}

// ---------------- weight and bias gradients: dW = dz^T h, db = dz^T 1 over row chunks
struct GemmJob {
  const float* dz;
  const float* h;
  float* wpart;    // [nch][O][I]
  float* bpart;    // [nch][O]
  int ldz, ldh, O, I;
};
struct GemmArgs {
  GemmJob job[NJOB];
  int order[NJOB];  // grid order of the jobs: the 128x128 layers first
  int nch, chunk;
};

// one workgroup per (job, chunk).  The chunk's dz and h rows pass through LDS in
// 32-row slabs (coalesced loads by all 256 threads, the next slab in flight
// while the current one feeds the MFMAs); wave w owns output rows 32w..32w+31
// and all (<= 4) 32-column blocks.
__global__ __launch_bounds__(256) void mlp_dw_kernel(GemmArgs g) {
  __shared__ float za[2][SLAB][LDT];
  __shared__ float hb[2][SLAB][LDT];
  const int j = g.order[blockIdx.x / g.nch], chunk = blockIdx.x % g.nch;
  const GemmJob J = g.job[j];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5;
  const int o = w * 32 + (lane & 31);
  const bool active = w * 32 < J.O;
  const int nib = (J.I + 31) / 32;
  const long long row0 = (long long)chunk * g.chunk;
  const int nslab = g.chunk / SLAB;
  // loader: thread tid fills columns c = tid & 127 of rows (tid >> 7) + 2i
  const int lc = tid & 127, lr = tid >> 7;
  const bool lz = lc < J.O, lh = lc < J.I;
  float rz[SLAB / 2], rh[SLAB / 2];
  auto load = [&](int slab) {
    const long long rb = row0 + (long long)slab * SLAB + lr;
#pragma unroll
    for (int i = 0; i < SLAB / 2; i++) {
      rz[i] = lz ? J.dz[(rb + 2 * i) * J.ldz + lc] : 0.f;
      rh[i] = lh ? J.h[(rb + 2 * i) * J.ldh + lc] : 0.f;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < SLAB / 2; i++) {
      za[buf][lr + 2 * i][lc] = rz[i];
      hb[buf][lr + 2 * i][lc] = rh[i];
    }
  };
  f32x16 acc[4];
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[q][r] = 0.f;
  float bsum = 0.f;
  load(0);
  stash(0);
  __syncthreads();
  for (int sl = 0; sl < nslab; sl++) {
    const int buf = sl & 1;
    if (sl + 1 < nslab) load(sl + 1);
    if (active) {
#pragma unroll
      for (int st = 0; st < SLAB / 2; st++) {
        const int r = 2 * st + hh;
        const float a = za[buf][r][o];
        bsum += a;
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (q < nib) acc[q] = mfma(a, hb[buf][r][q * 32 + (lane & 31)], acc[q]);
      }
    }
    if (sl + 1 < nslab) stash(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  const bool ok_o = o < J.O;
  bsum += __shfl_xor(bsum, 32, 64);
  if (hh == 0 && ok_o) J.bpart[(long long)chunk * J.O + o] = bsum;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int i = q * 32 + (lane & 31);
    if (q >= nib || i >= J.I) continue;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int oo = w * 32 + crow(r, lane);
      if (oo < J.O) J.wpart[((long long)chunk * J.O + oo) * J.I + i] = acc[q][r];
    }
  }
}

// ---------------- gradient assembly, norm partials, log_std, log row, counters
struct Seg {
  const float* src;  // chunk partials: element e of chunk c at src[c * n + e]
  int n, dst, first;
};
struct ReduceArgs {
  Seg seg[NSEG];
  int total, nch;
  float* grad;
  float* npart;
  const float* lpart;
  int ntiles, B, off_ls;
  const float* ls;
  float ent_coef, vf_coef;
  float* log;
  long long* mb_counter;
  long long* row_counter;
};

__global__ __launch_bounds__(256) void mlp_reduce_kernel(ReduceArgs a) {
  __shared__ float red[4];
  __shared__ float tsum[8];
  const int e = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (blockIdx.x == 0) {  // loss partials over the tiles: wave w sums q = w and q = w + 4
    float v0 = 0.f, v1 = 0.f;
    for (int t = lane; t < a.ntiles; t += 64) {
      v0 += a.lpart[(long long)t * LPART + wid];
      v1 += a.lpart[(long long)t * LPART + wid + 4];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      v0 += __shfl_xor(v0, off, 64);
      v1 += __shfl_xor(v1, off, 64);
    }
    if (lane == 0) { tsum[wid] = v0; tsum[wid + 4] = v1; }
    __syncthreads();
  }
  float g2 = 0.f;
  if (e < a.total) {
    int q = 0;
    for (int k = 1; k < NSEG; k++)
      if (e >= a.seg[k].first) q = k;
    const Seg S = a.seg[q];
    const int el = e - S.first;
    // eight independent partial sums keep eight loads in flight (fixed order)
    float p8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int c = 0;
    for (; c + 8 <= a.nch; c += 8) {
#pragma unroll
      for (int u = 0; u < 8; u++) p8[u] += S.src[(long long)(c + u) * S.n + el];
    }
    for (; c < a.nch; c++) p8[c & 7] += S.src[(long long)c * S.n + el];
    const float s = ((p8[0] + p8[1]) + (p8[2] + p8[3])) + ((p8[4] + p8[5]) + (p8[6] + p8[7]));
    a.grad[S.dst + el] = s;
    g2 = s * s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // d loss / d log_std_j = sum glp (z^2 - 1) - ent_coef
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const float gl = tsum[4 + j] - a.ent_coef;
      a.grad[a.off_ls + j] = gl;
      g2 += gl * gl;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) g2 += __shfl_xor(g2, off, 64);
  if (lane == 0) red[wid] = g2;
  __syncthreads();
  if (threadIdx.x != 0) return;
  a.npart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (blockIdx.x != 0) return;
  const float invB = 1.f / float(a.B);
  const float pg = tsum[0] * invB, vf = tsum[1] * invB;
  const float ent = -(3.f * (0.5f + HALF_LOG_2PI) + a.ls[0] + a.ls[1] + a.ls[2]);
  const long long row = *a.row_counter;
  float* L = a.log + row * 6;
  L[0] = pg + a.ent_coef * ent + a.vf_coef * vf;
  L[1] = pg;
  L[2] = vf;
  L[3] = ent;
  L[4] = tsum[2] * invB;
  L[5] = tsum[3] * invB;
  *a.row_counter = row + 1;
  *a.mb_counter = *a.mb_counter + 1;
}

}  // namespace

long long mlp_workspace_bytes(int B) {
  long long n = 0;
  carve(nullptr, B, &n);
  return n * 4;
}

int launch_mlp_step(const MlpStepArgs& A, hipStream_t s) {
  const int B = A.B;
  if (B < 256 || B % 256 || B > 16384 || (A.in_dim != 15 && A.in_dim != 56)) return -2;
  if (A.ws_bytes < mlp_workspace_bytes(B)) return -3;
  const Workspace w = carve(A.ws, B, nullptr);
  const int ntiles = B / ROWS, nch = n_chunks(B);
  if (A.phase == 2) {  // clip + AdamW only: the clip norm from the (all-reduced) flat gradient itself
    AdamWArgs o{A.params, A.grad, A.exp_avg, A.exp_avg_sq, A.n_params, A.lr, A.step, A.coef, A.beta1, A.beta2,
                A.weight_decay, float(A.beta2), float(1.0 - A.beta1), float(1.0 - A.beta2), float(A.eps),
                float(A.max_norm), nullptr, 0};
    if (launch_adamw_clip(o, s)) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }

  TileArgs t;
  t.P = A.params;
  for (int i = 0; i < MLP_NSLOTS; i++) t.off[i] = A.off[i];
  t.obs = A.obs; t.actions = A.actions; t.old_logp = A.old_logp; t.adv = A.adv; t.returns = A.returns;
  t.perm = A.perm; t.mb_counter = A.mb_counter; t.clip = A.clip;
  t.B = B; t.normalize = A.normalize; t.vf_coef = A.vf_coef; t.w = w; t.adv_stats = A.adv_stats;
  t.n = 0; t.noise = nullptr; t.obs_copy = t.act_out = t.act_clipped = t.values_out = t.logp_out = nullptr;
  t.obs_direct = A.obs_direct;
  if (A.in_dim == 15)
    hipLaunchKernelGGL((mlp_tile_kernel<true, 15>), dim3(ntiles), dim3(T1), 0, s, t);
  else
    hipLaunchKernelGGL((mlp_tile_kernel<true, 56>), dim3(ntiles), dim3(T1), 0, s, t);

  // weight/bias-gradient jobs, in flat-gradient segment order
  GemmArgs g;
  ReduceArgs r;
  int nj = 0, ns = 0, total = 0;
  float* wp = w.wpart;
  float* bp = w.bpart;
  auto add_job = [&](const float* dz, int ldz, int O, const float* h, int ldh, int I, int wdst, int bdst) {
    GemmJob& J = g.job[nj++];
    J.dz = dz; J.ldz = ldz; J.O = O; J.h = h; J.ldh = ldh; J.I = I; J.wpart = wp; J.bpart = bp;
    Seg& SW = r.seg[ns++];
    SW.src = wp; SW.n = O * I; SW.dst = wdst; SW.first = total; total += O * I;
    Seg& SB = r.seg[ns++];
    SB.src = bp; SB.n = O; SB.dst = bdst; SB.first = total; total += O;
    wp += (long long)nch * O * I;
    bp += (long long)nch * O;
  };
  for (int tr = 0; tr < 2; tr++)
    for (int l = 0; l < 4; l++)
      add_job(w.dz[tr][l], HID, HID, l ? w.h[tr][l - 1] : w.x, l ? HID : (A.in_dim <= 16 ? 32 : 64),
              l ? HID : A.in_dim,
              A.off[(tr ? MLP_VF_W0 : MLP_PI_W0) + l], A.off[(tr ? MLP_VF_B0 : MLP_PI_B0) + l]);
  add_job(w.dhead, 4, 3, w.h[0][3], HID, HID, A.off[MLP_WA], A.off[MLP_BA]);
  add_job(w.dhead + 3, 4, 1, w.h[1][3], HID, HID, A.off[MLP_WV], A.off[MLP_BV]);
  {  // grid order: the six 128x128 layers, then the input layers and the heads
    const int order[NJOB] = {1, 2, 3, 5, 6, 7, 0, 4, 8, 9};
    for (int q = 0; q < NJOB; q++) g.order[q] = order[q];
  }
  g.nch = nch;
  g.chunk = B / nch;
  hipLaunchKernelGGL(mlp_dw_kernel, dim3(NJOB * nch), dim3(256), 0, s, g);

  r.total = total; r.nch = nch;
  r.grad = A.grad; r.npart = w.npart; r.lpart = w.lpart; r.ntiles = ntiles; r.B = B; r.off_ls = A.off[MLP_LS];
  r.ls = A.params + A.off[MLP_LS]; r.ent_coef = A.ent_coef; r.vf_coef = A.vf_coef; r.log = A.log;
  r.mb_counter = A.mb_counter; r.row_counter = A.row_counter;
  const int nred = (total + 255) / 256;
  if (nred > 4096) return -4;
  hipLaunchKernelGGL(mlp_reduce_kernel, dim3(nred), dim3(256), 0, s, r);
  if (A.phase == 1) return hipGetLastError() == hipSuccess ? 0 : -1;  // the caller reduces the gradient first

  AdamWArgs o{A.params, A.grad, A.exp_avg, A.exp_avg_sq, A.n_params, A.lr, A.step, A.coef, A.beta1, A.beta2,
              A.weight_decay, float(A.beta2), float(1.0 - A.beta1), float(1.0 - A.beta2), float(A.eps),
              float(A.max_norm), w.npart, nred};
  if (launch_adamw_clip(o, s)) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_mlp_act(const MlpActArgs& A, hipStream_t s) {
  if (A.n <= 0) return 0;
  if (A.in_dim != 15 && A.in_dim != 56) return -2;
  TileArgs t{};
  t.P = A.params;
  for (int i = 0; i < MLP_NSLOTS; i++) t.off[i] = A.off[i];
  t.obs = A.obs; t.n = A.n; t.noise = A.noise; t.obs_copy = A.obs_copy; t.act_out = A.actions;
  t.act_clipped = A.clipped; t.values_out = A.values; t.logp_out = A.log_prob;
  if (A.in_dim == 15)
    hipLaunchKernelGGL((mlp_tile_kernel<false, 15>), dim3((A.n + ROWS - 1) / ROWS), dim3(T1), 0, s, t);
  else
    hipLaunchKernelGGL((mlp_tile_kernel<false, 56>), dim3((A.n + ROWS - 1) / ROWS), dim3(T1), 0, s, t);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
