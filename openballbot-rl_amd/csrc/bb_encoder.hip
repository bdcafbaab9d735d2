// bb_encoder.hip -- the frozen depth-image encoder of the camera policy, fused
// (SURVEY.md §8 F2).  The reference's rgbd branch with a pretrained encoder
// (ballbot_rl/encoders/models.py:6-54, loaded frozen by policies/mlp_policy.py:51-125):
//   Conv2d(1->32, k3 s2 p1) BatchNorm2d LeakyReLU  64x64 -> 32x32
//   Conv2d(32->32, k3 s2 p1) BatchNorm2d LeakyReLU 32x32 -> 16x16
//   Flatten (C, H, W) -> Linear(8192 -> 20) BatchNorm1d Tanh
// The weights are frozen, but SB3's policy.train() puts the BatchNorms in train
// mode during the update: each forward normalises with the batch's statistics
// (biased variance) and moves the running statistics (momentum 0.1, unbiased
// variance); in eval mode (the rollout) the running statistics normalise.
// Nothing downstream needs gradients through it.
//
// Launches per camera (n images):
//   train: conv1_stats -> bn_finish(1) -> conv2 -> bn_finish(2) -> linear -> head
//   eval:                bn_finish(1) -> conv2 -> bn_finish(2) -> linear -> head
// conv1 is recomputed where it is consumed (9 MACs per output): conv1_stats only
// accumulates its per-channel sums, conv2 rebuilds 16 channels at a time in LDS.
// conv2 is an implicit GEMM on v_mfma_f32_32x32x2_f32 (M = 32 output positions,
// N = 32 channels, K = 288 taps x channels); the linear layer is a 32-image x
// 32-output (20 used) MFMA GEMM over K = 8192.  Batch statistics accumulate in
// fp64.  fp32 arithmetic as the reference; only summation orders differ from
// MIOpen/PyTorch (tests/test_gpu_render.py: test_fused_encoder_matches_torch).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "bb_encoder.h"

namespace bb {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int IH = 64, IW = 64;     // input depth image
constexpr int C1 = 32, H1 = 32;     // conv1 output channels / side
constexpr int H2 = 16;              // conv2 output side
constexpr int K2 = C1 * 9;          // conv2 reduction length
constexpr int FL = C1 * H2 * H2;    // flattened conv2 output (8192)
constexpr int NZ = 20;              // encoder output features
constexpr int CS = H1 * H1 + 1;     // LDS channel stride of the conv1 tile (odd: lane halves hit other banks)
constexpr float SLOPE = 0.01f;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ float leaky(float z) { return z > 0.f ? z : z * SLOPE; }

// conv1 output (pre-BN) at channel oc, position (oy, ox) from the LDS image
__device__ __forceinline__ float conv1_at(const float (*x)[IW], const float* w1, float b1, int oy, int ox) {
  float v = b1;
#pragma unroll
  for (int ky = 0; ky < 3; ky++) {
    const int iy = 2 * oy + ky - 1;
#pragma unroll
    for (int kx = 0; kx < 3; kx++) {
      const int ix = 2 * ox + kx - 1;
      const float xv = (iy >= 0 && ix >= 0) ? x[iy][ix] : 0.f;  // iy, ix <= 63 always
      v = fmaf(w1[ky * 3 + kx], xv, v);
    }
  }
  return v;
}

__device__ __forceinline__ void stage_image(float (*x)[IW], const float* img) {
  for (int e = threadIdx.x; e < IH * IW / 4; e += 256)
    reinterpret_cast<float4*>(&x[0][0])[e] = reinterpret_cast<const float4*>(img)[e];
}

// ---- 1. conv1 batch statistics: one workgroup per 8 images; thread (oc, group)
__global__ __launch_bounds__(256) void conv1_stats_kernel(EncArgs a) {
  __shared__ __attribute__((aligned(16))) float x[IH][IW];
  __shared__ double red[8][C1][2];
  const int t = threadIdx.x, oc = t & 31, g = t >> 5;
  float w1[9];
#pragma unroll
  for (int k = 0; k < 9; k++) w1[k] = a.p.w1[oc * 9 + k];
  const float b1 = a.p.b1[oc];
  double s = 0.0, s2 = 0.0;
  for (int i = 0; i < 8; i++) {
    const long long b = (long long)blockIdx.x * 8 + i;
    if (b >= a.n) break;
    __syncthreads();
    stage_image(x, a.images + b * a.image_stride);
    __syncthreads();
    float fs = 0.f, fs2 = 0.f;
    for (int q = 0; q < H1 * H1 / 8; q++) {
      const int pos = g + 8 * q;
      const float v = conv1_at(x, w1, b1, pos >> 5, pos & 31);
      fs += v;
      fs2 += v * v;
    }
    s += fs;
    s2 += fs2;
  }
  red[g][oc][0] = s;
  red[g][oc][1] = s2;
  __syncthreads();
  if (t < 2 * C1) {
    const int c = t >> 1, k = t & 1;
    double v = 0.0;
    for (int gg = 0; gg < 8; gg++) v += red[gg][c][k];
    a.ws.part1[((long long)blockIdx.x * C1 + c) * 2 + k] = v;
  }
}

// ---- 2. BN finish: batch (train) or running (eval) statistics -> scale/shift
// (and, in train mode, the running-statistics update torch's BatchNorm makes)
__global__ __launch_bounds__(256) void bn_finish_kernel(const double* part, int nparts, long long count, int C,
                                                        const float* gamma, const float* beta, float* rmean,
                                                        float* rvar, long long* nbt, int train, float momentum,
                                                        float eps, float* scale_shift) {
  const int c = threadIdx.x;
  if (c >= C) return;
  float mean, var;
  if (train) {
    double s = 0.0, s2 = 0.0;
    for (int p = 0; p < nparts; p++) {
      s += part[((long long)p * C + c) * 2];
      s2 += part[((long long)p * C + c) * 2 + 1];
    }
    const double m = s / double(count);
    const double v = fmax(s2 / double(count) - m * m, 0.0);
    mean = float(m);
    var = float(v);
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * float(v * double(count) / double(count > 1 ? count - 1 : 1));
    if (c == 0 && nbt) *nbt += 1;
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  const float sc = gamma[c] / sqrtf(var + eps);
  scale_shift[c] = sc;
  scale_shift[C + c] = beta[c] - mean * sc;
}

// ---- 3. conv2 as an implicit GEMM; grid-stride over images.  Per image: the
// image in LDS, then twice (input channels 0-15, 16-31): conv1 + BN1 + LeakyReLU
// of those channels into LDS, and 72 MFMA steps per 32-position block.
// Wave w owns position blocks 2w, 2w+1 (rows 4w..4w+3 of the 16x16 output).
__global__ __launch_bounds__(256) void conv2_kernel(EncArgs a) {
  __shared__ __attribute__((aligned(16))) float x[IH][IW];
  __shared__ float a1[16 * CS];       // 16 channels of the activated conv1 output
  __shared__ float w2t[K2][C1];       // conv2 weights, [ic*9 + tap][oc]
  __shared__ float ss1[2 * C1];
  __shared__ double red[4][C1][2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, hh = lane >> 5, oc = lane & 31;
  for (int e = t; e < K2 * C1; e += 256) {
    const int o = e / K2, k = e % K2;
    w2t[k][o] = a.p.w2[e];
  }
  if (t < 2 * C1) ss1[t] = a.ws.ss1[t];
  const float b2 = a.p.b2[oc];
  double s = 0.0, s2 = 0.0;
  // this lane's two output positions (A rows) in its wave's blocks
  int py[2], px[2];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int pos = (2 * w + q) * 32 + (lane & 31);
    py[q] = pos >> 4;
    px[q] = pos & 15;
  }
  for (long long b = blockIdx.x; b < a.n; b += gridDim.x) {
    __syncthreads();
    stage_image(x, a.images + b * a.image_stride);
    f32x16 acc[2];
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[q][r] = b2;
    for (int half = 0; half < 2; half++) {
      __syncthreads();  // image staged / previous half consumed
      for (int icl = 0; icl < 16; icl++) {  // the channel is uniform: its weights are scalar loads
        const int ic = 16 * half + icl;
        float w1[9];
#pragma unroll
        for (int k = 0; k < 9; k++) w1[k] = a.p.w1[ic * 9 + k];
        const float b1 = a.p.b1[ic], sc = ss1[ic], sh = ss1[C1 + ic];
#pragma unroll
        for (int j = 0; j < H1 * H1 / 256; j++) {
          const int pos = t + 256 * j;
          a1[icl * CS + pos] = leaky(fmaf(conv1_at(x, w1, b1, pos >> 5, pos & 31), sc, sh));
        }
      }
      __syncthreads();
      // K order: step (icp, tap): lane half hh takes input channel 2 icp + hh
      for (int icp = 0; icp < 8; icp++) {
        const int icl = 2 * icp + hh, ic = 16 * half + icl;
        const float* ach = a1 + icl * CS;
#pragma unroll
        for (int tap = 0; tap < 9; tap++) {
          const int ky = tap / 3, kx = tap % 3;
          const float bw = w2t[ic * 9 + tap][oc];
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const int iy = 2 * py[q] + ky - 1, ix = 2 * px[q] + kx - 1;
            const float av = (iy >= 0 && ix >= 0) ? ach[iy * H1 + ix] : 0.f;
            acc[q] = mfma(av, bw, acc[q]);
          }
        }
      }
    }
    // raw conv2 output, flattened (C, H, W): column = channel, rows = positions
    float* out = a.ws.out2 + b * FL;
#pragma unroll
    for (int q = 0; q < 2; q++) {
      float fs = 0.f, fs2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int pos = (2 * w + q) * 32 + crow(r, lane);
        const float v = acc[q][r];
        out[oc * (H2 * H2) + pos] = v;
        fs += v;
        fs2 += v * v;
      }
      s += fs;
      s2 += fs2;
    }
  }
  if (a.train) {
    s += __shfl_xor(s, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (hh == 0) { red[w][oc][0] = s; red[w][oc][1] = s2; }
    __syncthreads();
    if (t < 2 * C1) {
      const int c = t >> 1, k = t & 1;
      a.ws.part2[((long long)blockIdx.x * C1 + c) * 2 + k] = (red[0][c][k] + red[1][c][k]) + (red[2][c][k] + red[3][c][k]);
    }
  }
}

// ---- 4. Linear(8192 -> 20) on BN2 + LeakyReLU(conv2): 32 images per workgroup,
// wave w sums K range [2048 w, 2048 w + 2048); the four partial tiles add in LDS
__global__ __launch_bounds__(256) void linear_kernel(EncArgs a) {
  __shared__ float tile[4][32][33];
  __shared__ float ss2[2 * C1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, hh = lane >> 5, r32 = lane & 31;
  if (t < 2 * C1) ss2[t] = a.ws.ss2[t];
  __syncthreads();
  const long long img = (long long)blockIdx.x * 32 + r32;
  const bool ok_img = img < a.n;
  const bool ok_j = r32 < NZ;
  const float* arow = a.ws.out2 + (ok_img ? img : 0) * FL + 4 * hh;
  const float* wrow = a.p.wl + (ok_j ? r32 : 0) * FL + 4 * hh;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  const int k0 = w * (FL / 4);
#pragma unroll 4
  for (int m = 0; m < FL / 4 / 8; m++) {
    const int k = k0 + 8 * m;
    const int c = (k + 4 * hh) >> 8;  // channel of these four features
    float4 av = *reinterpret_cast<const float4*>(arow + k);
    float4 bv = *reinterpret_cast<const float4*>(wrow + k);
    const float sc = ss2[c], sh = ss2[C1 + c];
    av.x = ok_img ? leaky(fmaf(av.x, sc, sh)) : 0.f;
    av.y = ok_img ? leaky(fmaf(av.y, sc, sh)) : 0.f;
    av.z = ok_img ? leaky(fmaf(av.z, sc, sh)) : 0.f;
    av.w = ok_img ? leaky(fmaf(av.w, sc, sh)) : 0.f;
    if (!ok_j) bv = make_float4(0.f, 0.f, 0.f, 0.f);
    acc = mfma(av.x, bv.x, acc);
    acc = mfma(av.y, bv.y, acc);
    acc = mfma(av.z, bv.z, acc);
    acc = mfma(av.w, bv.w, acc);
  }
  // C layout: column = output feature j, rows = images
#pragma unroll
  for (int r = 0; r < 16; r++) tile[w][crow(r, lane)][r32] = acc[r];
  __syncthreads();
  for (int e = t; e < 32 * NZ; e += 256) {
    const int i = e / NZ, j = e % NZ;
    const long long im = (long long)blockIdx.x * 32 + i;
    if (im >= a.n) continue;
    a.ws.z[im * NZ + j] = ((tile[0][i][j] + tile[1][i][j]) + (tile[2][i][j] + tile[3][i][j])) + a.p.bl[j];
  }
}

// ---- 5. BatchNorm1d(20) + Tanh -> features; one 1024-thread workgroup
__global__ __launch_bounds__(1024) void head_kernel(EncArgs a) {
  __shared__ double red[32][NZ][2];
  __shared__ float sc[NZ], sh[NZ];
  const int t = threadIdx.x, lane = t & 31, grp = t >> 5;  // 32 groups of 32 threads
  if (a.train) {
    // thread (grp, lane): channel j = lane (< 20), images grp, grp + 32, ...
    double s = 0.0, s2 = 0.0;
    if (lane < NZ)
      for (long long i = grp; i < a.n; i += 32) {
        const double v = a.ws.z[i * NZ + lane];
        s += v;
        s2 += v * v;
      }
    if (lane < NZ) { red[grp][lane][0] = s; red[grp][lane][1] = s2; }
    __syncthreads();
    if (t < NZ) {
      double S = 0.0, S2 = 0.0;
      for (int g = 0; g < 32; g++) { S += red[g][t][0]; S2 += red[g][t][1]; }
      const double cnt = double(a.n);
      const double m = S / cnt, v = fmax(S2 / cnt - m * m, 0.0);
      a.p.rm3[t] = (1.f - a.momentum) * a.p.rm3[t] + a.momentum * float(m);
      a.p.rv3[t] = (1.f - a.momentum) * a.p.rv3[t] + a.momentum * float(v * cnt / (a.n > 1 ? cnt - 1.0 : 1.0));
      if (t == 0 && a.p.nbt3) *a.p.nbt3 += 1;
      const float s_ = a.p.g3[t] / sqrtf(float(v) + a.eps);
      sc[t] = s_;
      sh[t] = a.p.be3[t] - float(m) * s_;
    }
  } else if (t < NZ) {
    const float s_ = a.p.g3[t] / sqrtf(a.p.rv3[t] + a.eps);
    sc[t] = s_;
    sh[t] = a.p.be3[t] - a.p.rm3[t] * s_;
  }
  __syncthreads();
  for (long long e = t; e < a.n * NZ; e += 1024) {
    const int j = int(e % NZ);
    a.out[(e / NZ) * a.out_stride + j] = tanhf(fmaf(a.ws.z[e], sc[j], sh[j]));
  }
}

EncWorkspace carve(float* base, long long n, long long* total) {
  EncWorkspace w;
  long long o = 0;
  auto take = [&](long long nfloats) { float* p = base ? base + o : nullptr; o += (nfloats + 63) & ~63LL; return p; };
  const long long g1 = (n + 7) / 8;
  w.part1 = reinterpret_cast<double*>(take(g1 * C1 * 2 * 2));
  w.part2 = reinterpret_cast<double*>(take(256LL * C1 * 2 * 2));
  w.ss1 = take(2 * C1);
  w.ss2 = take(2 * C1);
  w.out2 = take(n * FL);
  w.z = take(n * NZ);
  if (total) *total = o;
  return w;
}

}  // namespace

long long encoder_workspace_bytes(long long n) {
  long long f = 0;
  carve(nullptr, n, &f);
  return f * 4;
}

int launch_encoder(EncArgs a, float* ws, hipStream_t s) {
  if (a.n <= 0) return 0;
  a.ws = carve(ws, a.n, nullptr);
  const int g1 = int((a.n + 7) / 8);
  const int g2 = int(a.n < 256 ? a.n : 256);
  if (a.train) hipLaunchKernelGGL(conv1_stats_kernel, dim3(g1), dim3(256), 0, s, a);
  hipLaunchKernelGGL(bn_finish_kernel, dim3(1), dim3(256), 0, s, (const double*)a.ws.part1, g1, a.n * H1 * H1, C1,
                     a.p.g1, a.p.be1, a.p.rm1, a.p.rv1, a.p.nbt1, a.train, a.momentum, a.eps, a.ws.ss1);
  hipLaunchKernelGGL(conv2_kernel, dim3(g2), dim3(256), 0, s, a);
  hipLaunchKernelGGL(bn_finish_kernel, dim3(1), dim3(256), 0, s, (const double*)a.ws.part2, g2, a.n * H2 * H2, C1,
                     a.p.g2, a.p.be2, a.p.rm2, a.p.rv2, a.p.nbt2, a.train, a.momentum, a.eps, a.ws.ss2);
  hipLaunchKernelGGL(linear_kernel, dim3(int((a.n + 31) / 32)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(head_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
