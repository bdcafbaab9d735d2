// bb_mlp.hip -- one PPO minibatch of the reference's proprio policy, fused
// (SURVEY.md §8 F1): forward of both 4x128 LeakyReLU trunks, the Gaussian and
// value heads, SB3 2.6.0's PPO loss and its gradients, the backward pass, the
// weight gradients, clip_grad_norm_ and AdamW -- five launches instead of the
// ~50 PyTorch/hipBLASLt launches of the autograd path.
//
// The policy (ballbot_rl/policies/mlp_policy.py:143-163, train.py:39-56):
//   f = obs (15 floats, sorted-key proprio)
//   pi: h1..h4 = leaky(h W^T + b), 15->128->128->128->128;  mean = h4 Wa^T + ba (3)
//   vf: the same trunk shape;                               value = h4 Wv^T + bv (1)
// The loss is bb_ppo.hip's (clipped surrogate, MSE value loss, entropy of a
// state-independent log_std); its per-sample gradient needs only the
// minibatch's advantage mean/std, which every tile recomputes (same order, so
// the same bits), so the gradient flows back through the tile that formed it.
//
// Launches (B = minibatch rows, tiles of 32 rows):
//   1. mlp_tile_kernel   B/32 workgroups x 4 waves.  Wave w owns columns
//      32w..32w+31 of every 128-wide layer; a layer is 64 (K=128) or 8 (K=16)
//      v_mfma_f32_32x32x2_f32 per wave with the layer input read from an LDS
//      tile (float4 per lane, k order permuted identically for A and B) and
//      W from L2.  Activations stay in registers in the MFMA C layout (h1..h4
//      of both trunks: 128 VGPRs) for the LeakyReLU backward; the heads and the
//      loss run on the VALU.  Backward: dh_l = dz_{l+1} W_l (MFMA again).
//      Layer inputs h_l and output gradients dz_{l+1} go to a workspace for
//      launch 2; bias gradients and loss terms leave as per-tile partials.
//   2. mlp_dw_kernel     dW_l = dz_{l+1}^T h_l as 32x32 MFMA blocks over
//      K = B/8 row chunks, one wave per (layer, block, chunk): 896 waves at
//      B = 8192.
//   3. mlp_reduce_kernel sums the chunk/tile partials in a fixed order into the
//      flat gradient buffer, g^2 per workgroup for the clip, the log row, and
//      advances the minibatch/log-row counters (graph replays).
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
constexpr int IN = 15;            // observation features
constexpr int XW = 32;            // workspace row width of the padded input
constexpr int ROWS = 32;          // rows per tile (the MFMA M)
constexpr int T1 = 256;           // threads per tile workgroup
constexpr int LDT = HID + 4;      // LDS row stride (floats): float4 rows, no bank conflicts
constexpr int LDX = IN + 2;       // input tile stride
constexpr int NCH = 8;            // K chunks of the weight-gradient GEMMs
constexpr int BPART = 2 * 4 * HID + 4;  // bias partials per tile: trunk biases, ba[3], bv
constexpr int LPART = 8;          // loss partials per tile: pg, vf, kl, cf, dls[3], -
constexpr int NJOB = 10;          // weight-gradient GEMMs: 2 trunks x 4 layers + 2 heads
constexpr int NSEG = 21;          // gradient segments (weights, biases, log_std)
constexpr float SLOPE = 0.01f;    // nn.LeakyReLU default negative_slope
constexpr float HALF_LOG_2PI = 0.91893853320467274f;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// C/D layout of the 32x32 f32 MFMA: column = lane & 31, row = crow(reg, lane)
__device__ __forceinline__ int crow(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ float leaky(float z) { return z > 0.f ? z : z * SLOPE; }

struct Workspace {
  float* x;           // [B][32] padded inputs
  float* h[2][4];     // [B][128] h1..h4 per trunk
  float* dz[2][4];    // [B][128] dL/dz of layers 0..3 per trunk
  float* dhead;       // [B][4] dL/dmean[3], dL/dvalue
  float* bpart;       // [B/32][BPART]
  float* lpart;       // [B/32][LPART]
  float* wpart;       // [NCH][weights]
  float* npart;       // [reduce workgroups]
};

Workspace carve(float* base, int B, long long* total_floats) {
  Workspace w;
  long long o = 0;
  auto take = [&](long long n) { float* p = base ? base + o : nullptr; o += (n + 63) & ~63LL; return p; };
  w.x = take((long long)B * XW);
  for (int t = 0; t < 2; t++)
    for (int l = 0; l < 4; l++) w.h[t][l] = take((long long)B * HID);
  for (int t = 0; t < 2; t++)
    for (int l = 0; l < 4; l++) w.dz[t][l] = take((long long)B * HID);
  w.dhead = take((long long)B * 4);
  w.bpart = take((long long)(B / ROWS) * BPART);
  w.lpart = take((long long)(B / ROWS) * LPART);
  w.wpart = take((long long)NCH * (2 * (HID * IN + 3 * HID * HID) + 4 * HID));
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
  int B, normalize;
  float vf_coef;
  Workspace w;
};

// block-wide sum over T1 threads, same order in every workgroup
__device__ float block_sum(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// store a wave's 32x32 C-layout block: rows of the tile, columns col0..col0+31
__device__ __forceinline__ void store_block(const f32x16& v, float* dst, int ld, int col, int lane) {
#pragma unroll
  for (int r = 0; r < 16; r++) dst[(long long)crow(r, lane) * ld + col] = v[r];
}

// a layer's output gradient: to the workspace (weight GEMMs) and its column
// sums over the tile (bias gradient partial)
__device__ __forceinline__ void dz_out(const f32x16& dz, const Workspace& w, int t, int l, int r0, int tile, int col,
                                       int lane) {
  store_block(dz, w.dz[t][l] + (long long)r0 * HID, HID, col, lane);
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; r++) s += dz[r];
  s += __shfl_xor(s, 32, 64);
  if (lane < 32) w.bpart[(long long)tile * BPART + t * 4 * HID + l * HID + col] = s;
}

__global__ __launch_bounds__(T1) void mlp_tile_kernel(TileArgs p) {
  __shared__ __attribute__((aligned(16))) float xs[2][ROWS][LDT];  // layer-input exchange tiles
  __shared__ float xin[ROWS][LDX];
  __shared__ float head[ROWS][4];  // dL/dmean[3], dL/dvalue
  __shared__ float hm[ROWS][4];    // mean[3], value
  __shared__ float red[4];
  __shared__ int idx[ROWS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5;
  const int col = w * 32 + (lane & 31);
  const int B = p.B, tile = blockIdx.x, r0 = tile * ROWS;
  const long long* perm = p.perm + (*p.mb_counter) * (long long)B;
  const float* P = p.P;

  // advantage normalisation over the minibatch (torch.std: unbiased)
  float amean = 0.f, ainv = 1.f;
  if (p.normalize && B > 1) {
    float s = 0.f;
    for (int i = tid; i < B; i += T1) s += p.adv[perm[i]];
    amean = block_sum(s, red) / float(B);
    float q = 0.f;
    for (int i = tid; i < B; i += T1) { const float d = p.adv[perm[i]] - amean; q += d * d; }
    ainv = 1.f / (sqrtf(block_sum(q, red) / float(B - 1)) + 1e-8f);
  }

  if (tid < ROWS) idx[tid] = (int)perm[r0 + tid];
  __syncthreads();
  for (int e = tid; e < ROWS * XW; e += T1) {
    const int r = e >> 5, c = e & 31;
    const float v = c < IN ? p.obs[(long long)idx[r] * IN + c] : 0.f;
    if (c < LDX) xin[r][c] = v;
    p.w.x[(long long)(r0 + r) * XW + c] = v;
  }
  __syncthreads();

  // ---------------- forward: both trunks, activations kept in C layout
  f32x16 hreg[2][4];
  int cur = 0;
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int ow = p.off[t ? MLP_VF_W0 : MLP_PI_W0], ob = p.off[t ? MLP_VF_B0 : MLP_PI_B0];
    {  // layer 0, K = 15 (padded to 16)
      f32x16 acc;
      const float bias = P[ob + col];
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = bias;
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const int k = 2 * s + hh;
        const float a = xin[lane & 31][k];
        const float b = k < IN ? P[ow + col * IN + k] : 0.f;
        acc = mfma(a, b, acc);
      }
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = leaky(acc[r]);
      hreg[t][0] = acc;
      store_block(acc, p.w.h[t][0] + (long long)r0 * HID, HID, col, lane);
      store_block(acc, &xs[cur][0][0], LDT, col, lane);
      __syncthreads();
    }
#pragma unroll
    for (int l = 1; l < 4; l++) {
      const float* W = P + p.off[(t ? MLP_VF_W0 : MLP_PI_W0) + l];
      f32x16 acc;
      const float bias = P[p.off[(t ? MLP_VF_B0 : MLP_PI_B0) + l] + col];
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = bias;
      const float* arow = &xs[cur][lane & 31][4 * hh];
      const float* wrow = W + col * HID + 4 * hh;
#pragma unroll 4
      for (int m = 0; m < HID / 8; m++) {
        const float4 a4 = *reinterpret_cast<const float4*>(arow + 8 * m);
        const float4 b4 = *reinterpret_cast<const float4*>(wrow + 8 * m);
        acc = mfma(a4.x, b4.x, acc);
        acc = mfma(a4.y, b4.y, acc);
        acc = mfma(a4.z, b4.z, acc);
        acc = mfma(a4.w, b4.w, acc);
      }
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = leaky(acc[r]);
      hreg[t][l] = acc;
      store_block(acc, p.w.h[t][l] + (long long)r0 * HID, HID, col, lane);
      store_block(acc, &xs[cur ^ 1][0][0], LDT, col, lane);
      cur ^= 1;
      __syncthreads();
    }
    // head on h4 (xs[cur]): thread (row tid>>3, part tid&7) sums 16 columns
    {
      const int r = tid >> 3, part = tid & 7;
      const float* hrow = &xs[cur][r][part * 16];
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
      if (t == 0) {
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
        if (t == 0) {
          hm[r][0] = s0 + P[p.off[MLP_BA]];
          hm[r][1] = s1 + P[p.off[MLP_BA] + 1];
          hm[r][2] = s2 + P[p.off[MLP_BA] + 2];
        } else {
          hm[r][3] = s0 + P[p.off[MLP_BV]];
        }
      }
    }
    __syncthreads();
  }

  // ---------------- loss (SB3 PPO.train, bb_ppo.hip) and head gradients: wave 0, lane = row
  if (w == 0) {
    const float c = *p.clip;
    const float* ls = P + p.off[MLP_LS];
    const float l0 = ls[0], l1 = ls[1], l2 = ls[2];
    const float inv_std[3] = {expf(-l0), expf(-l1), expf(-l2)};
    const float lp_const = -(l0 + l1 + l2) - 3.f * HALF_LOG_2PI;
    const float invB = 1.f / float(B);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float gh[4] = {0, 0, 0, 0};
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
#pragma unroll
      for (int j = 0; j < 4; j++) gh[j] += __shfl_xor(gh[j], off, 64);
    }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 7; q++) p.w.lpart[(long long)tile * LPART + q] = acc[q];
      p.w.lpart[(long long)tile * LPART + 7] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; j++) p.w.bpart[(long long)tile * BPART + 2 * 4 * HID + j] = gh[j];
    }
  }
  __syncthreads();

  // ---------------- backward through both trunks
#pragma unroll
  for (int t = 0; t < 2; t++) {
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
        dz[r] = hreg[t][3][r] > 0.f ? d : d * SLOPE;
      }
    }
#pragma unroll
    for (int l = 3; l >= 1; l--) {
      dz_out(dz, p.w, t, l, r0, tile, col, lane);
      store_block(dz, &xs[cur][0][0], LDT, col, lane);
      __syncthreads();
      const float* W = P + p.off[(t ? MLP_VF_W0 : MLP_PI_W0) + l];
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = 0.f;
      const float* arow = &xs[cur][lane & 31][4 * hh];
      const float* wcol = W + 4 * hh * HID + col;
#pragma unroll 4
      for (int m = 0; m < HID / 8; m++) {
        const float4 a4 = *reinterpret_cast<const float4*>(arow + 8 * m);
        const float* wp = wcol + 8 * m * HID;
        acc = mfma(a4.x, wp[0], acc);
        acc = mfma(a4.y, wp[HID], acc);
        acc = mfma(a4.z, wp[2 * HID], acc);
        acc = mfma(a4.w, wp[3 * HID], acc);
      }
#pragma unroll
      for (int r = 0; r < 16; r++) dz[r] = hreg[t][l - 1][r] > 0.f ? acc[r] : acc[r] * SLOPE;
      cur ^= 1;
    }
    dz_out(dz, p.w, t, 0, r0, tile, col, lane);
  }
}

// ---------------- weight gradients: dW = dz^T h over row chunks
struct GemmJob {
  const float* dz;
  const float* h;
  float* part;     // [NCH][O][I]
  int ldz, ldh, O, I, nob, nib, first;
};
struct GemmArgs {
  GemmJob job[NJOB];
  int nunits, chunk;
};

constexpr int PF = 16;  // MFMA steps per prefetch batch

__global__ __launch_bounds__(256) void mlp_dw_kernel(GemmArgs g) {
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit >= g.nunits) return;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  int j = 0;
#pragma unroll
  for (int q = 1; q < NJOB; q++)
    if (unit >= g.job[q].first) j = q;
  const GemmJob J = g.job[j];
  const int u = unit - J.first, nblk = J.nob * J.nib;
  const int chunk = u / nblk, ob = (u % nblk) / J.nib, ib = u % J.nib;
  const int o = ob * 32 + (lane & 31), i = ib * 32 + (lane & 31);
  const bool ok_o = o < J.O, ok_i = i < J.I;
  const long long rb = (long long)chunk * g.chunk + hh;
  const float* zp = J.dz + rb * J.ldz + (ok_o ? o : 0);
  const float* hp = J.h + rb * J.ldh + (ok_i ? i : 0);
  const long long zs = 2LL * J.ldz, hs = 2LL * J.ldh;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  float a[PF], b[PF];
#pragma unroll
  for (int s = 0; s < PF; s++) { a[s] = zp[s * zs]; b[s] = hp[s * hs]; }
  const int steps = g.chunk / 2;
  for (int s0 = 0; s0 < steps; s0 += PF) {
    float an[PF], bn[PF];
    const bool more = s0 + PF < steps;
#pragma unroll
    for (int s = 0; s < PF; s++) {
      an[s] = more ? zp[(s0 + PF + s) * zs] : 0.f;
      bn[s] = more ? hp[(s0 + PF + s) * hs] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < PF; s++) acc = mfma(ok_o ? a[s] : 0.f, ok_i ? b[s] : 0.f, acc);
#pragma unroll
    for (int s = 0; s < PF; s++) { a[s] = an[s]; b[s] = bn[s]; }
  }
  if (!ok_i) return;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int oo = ob * 32 + crow(r, lane);
    if (oo < J.O) J.part[((long long)chunk * J.O + oo) * J.I + i] = acc[r];
  }
}

// ---------------- gradient assembly, norm partials, log row, counters
struct Seg {
  const float* src;  // partials: element e of partial c at src[c * stride + e]
  int n, count, stride, dst, first;
  float add;
};
struct ReduceArgs {
  Seg seg[NSEG];
  int total;
  float* grad;
  float* npart;
  const float* lpart;
  int ntiles, B;
  const float* ls;
  float ent_coef, vf_coef;
  float* log;
  long long* mb_counter;
  long long* row_counter;
};

__global__ __launch_bounds__(256) void mlp_reduce_kernel(ReduceArgs a) {
  __shared__ float red[4][4];
  const int e = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float g2 = 0.f;
  if (e < a.total) {
    int q = 0;
    for (int k = 1; k < NSEG; k++)
      if (e >= a.seg[k].first) q = k;
    const Seg S = a.seg[q];
    const int el = e - S.first;
    float s = 0.f;
    for (int c = 0; c < S.count; c++) s += S.src[(long long)c * S.stride + el];
    s += S.add;
    a.grad[S.dst + el] = s;
    g2 = s * s;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) g2 += __shfl_xor(g2, off, 64);
  if (lane == 0) red[0][wid] = g2;
  __syncthreads();
  if (threadIdx.x == 0) a.npart[blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  if (blockIdx.x != 0) return;
  // log row: wave q < 4 sums loss partial q over the tiles
  float v = 0.f;
  for (int t = lane; t < a.ntiles; t += 64) v += a.lpart[(long long)t * LPART + wid];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();
  if (lane == 0) red[1][wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float invB = 1.f / float(a.B);
    const float pg = red[1][0] * invB, vf = red[1][1] * invB;
    const float ent = -(3.f * (0.5f + HALF_LOG_2PI) + a.ls[0] + a.ls[1] + a.ls[2]);
    const long long row = *a.row_counter;
    float* L = a.log + row * 6;
    L[0] = pg + a.ent_coef * ent + a.vf_coef * vf;
    L[1] = pg;
    L[2] = vf;
    L[3] = ent;
    L[4] = red[1][2] * invB;
    L[5] = red[1][3] * invB;
    *a.row_counter = row + 1;
    *a.mb_counter = *a.mb_counter + 1;
  }
}

}  // namespace

long long mlp_workspace_bytes(int B) {
  long long n = 0;
  carve(nullptr, B, &n);
  return n * 4;
}

int launch_mlp_step(const MlpStepArgs& A, hipStream_t s) {
  const int B = A.B;
  if (B < 256 || B % ROWS || (B / NCH) % (2 * PF)) return -2;
  if (A.ws_bytes < mlp_workspace_bytes(B)) return -3;
  const Workspace w = carve(A.ws, B, nullptr);
  const int ntiles = B / ROWS;

  TileArgs t;
  t.P = A.params;
  for (int i = 0; i < MLP_NSLOTS; i++) t.off[i] = A.off[i];
  t.obs = A.obs; t.actions = A.actions; t.old_logp = A.old_logp; t.adv = A.adv; t.returns = A.returns;
  t.perm = A.perm; t.mb_counter = A.mb_counter; t.clip = A.clip;
  t.B = B; t.normalize = A.normalize; t.vf_coef = A.vf_coef; t.w = w;
  hipLaunchKernelGGL(mlp_tile_kernel, dim3(ntiles), dim3(T1), 0, s, t);

  // weight-gradient jobs, in flat-gradient segment order
  GemmArgs g;
  int nunits = 0, nj = 0;
  auto add_job = [&](const float* dz, int ldz, int O, const float* h, int ldh, int I, float* part) {
    GemmJob& J = g.job[nj++];
    J.dz = dz; J.ldz = ldz; J.O = O; J.h = h; J.ldh = ldh; J.I = I; J.part = part;
    J.nob = (O + 31) / 32; J.nib = (I + 31) / 32; J.first = nunits;
    nunits += J.nob * J.nib * NCH;
  };
  float* wp = w.wpart;
  const float* wbase[NJOB];
  int wsize[NJOB], wdst[NJOB];
  for (int tr = 0; tr < 2; tr++)
    for (int l = 0; l < 4; l++) {
      const int I = l ? HID : IN;
      wbase[nj] = wp; wsize[nj] = HID * I; wdst[nj] = A.off[(tr ? MLP_VF_W0 : MLP_PI_W0) + l];
      add_job(w.dz[tr][l], HID, HID, l ? w.h[tr][l - 1] : w.x, l ? HID : XW, I, wp);
      wp += (long long)NCH * HID * I;
    }
  wbase[nj] = wp; wsize[nj] = 3 * HID; wdst[nj] = A.off[MLP_WA];
  add_job(w.dhead, 4, 3, w.h[0][3], HID, HID, wp);
  wp += (long long)NCH * 3 * HID;
  wbase[nj] = wp; wsize[nj] = HID; wdst[nj] = A.off[MLP_WV];
  add_job(w.dhead + 3, 4, 1, w.h[1][3], HID, HID, wp);
  g.nunits = nunits;
  g.chunk = B / NCH;
  hipLaunchKernelGGL(mlp_dw_kernel, dim3((nunits + 3) / 4), dim3(256), 0, s, g);

  ReduceArgs r;
  int total = 0, ns = 0;
  auto add_seg = [&](const float* src, int n, int count, int stride, int dst, float add) {
    Seg& S = r.seg[ns++];
    S.src = src; S.n = n; S.count = count; S.stride = stride; S.dst = dst; S.first = total; S.add = add;
    total += n;
  };
  for (int j = 0; j < NJOB; j++) add_seg(wbase[j], wsize[j], NCH, wsize[j], wdst[j], 0.f);
  for (int tr = 0; tr < 2; tr++)
    for (int l = 0; l < 4; l++)
      add_seg(w.bpart + tr * 4 * HID + l * HID, HID, ntiles, BPART, A.off[(tr ? MLP_VF_B0 : MLP_PI_B0) + l], 0.f);
  add_seg(w.bpart + 2 * 4 * HID, 3, ntiles, BPART, A.off[MLP_BA], 0.f);
  add_seg(w.bpart + 2 * 4 * HID + 3, 1, ntiles, BPART, A.off[MLP_BV], 0.f);
  add_seg(w.lpart + 4, 3, ntiles, LPART, A.off[MLP_LS], -A.ent_coef);
  r.total = total;
  r.grad = A.grad; r.npart = w.npart; r.lpart = w.lpart; r.ntiles = ntiles; r.B = B;
  r.ls = A.params + A.off[MLP_LS]; r.ent_coef = A.ent_coef; r.vf_coef = A.vf_coef; r.log = A.log;
  r.mb_counter = A.mb_counter; r.row_counter = A.row_counter;
  const int nred = (total + 255) / 256;
  if (nred > 4096) return -4;
  hipLaunchKernelGGL(mlp_reduce_kernel, dim3(nred), dim3(256), 0, s, r);

  AdamWArgs o{A.params, A.grad, A.exp_avg, A.exp_avg_sq, A.n_params, A.lr, A.step, A.coef, A.beta1, A.beta2,
              A.weight_decay, float(A.beta2), float(1.0 - A.beta1), float(1.0 - A.beta2), float(A.eps),
              float(A.max_norm), w.npart, nred};
  if (launch_adamw_clip(o, s)) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
