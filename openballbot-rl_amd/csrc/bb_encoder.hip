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
//   train: conv1_moments -> bn1_moments -> conv2 -> bn_finish(2) -> linear -> head
//   eval:                   bn_finish(1) -> conv2 -> bn_finish(2) -> linear -> head
// conv1 is linear in its 3x3 input window, so its batch statistics come from
// the windows' 9 means and 45 products (conv1_moments); conv2 recomputes conv1
// where it consumes it (9 MACs per output), 16 channels at a time in LDS.
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

// image b of the batch: row index[b] of the image array when an index is given
__device__ __forceinline__ const float* image_of(const EncArgs& a, long long b) {
  return a.images + (a.index ? a.index[b] : b) * a.image_stride;
}

__device__ __forceinline__ void stage_image(float (*x)[IW], const float* img) {
  for (int e = threadIdx.x; e < IH * IW / 4; e += 256)
    reinterpret_cast<float4*>(&x[0][0])[e] = reinterpret_cast<const float4*>(img)[e];
}

// the 3x3 stride-2 input window of conv1 output position pos (zero padded)
__device__ __forceinline__ void window(const float (*x)[IW], int pos, float (&xv)[9]) {
  const int oy = pos >> 5, ox = pos & 31;
#pragma unroll
  for (int ky = 0; ky < 3; ky++)
#pragma unroll
    for (int kx = 0; kx < 3; kx++) {
      const int iy = 2 * oy + ky - 1, ix = 2 * ox + kx - 1;
      xv[ky * 3 + kx] = (iy >= 0 && ix >= 0) ? x[iy][ix] : 0.f;  // iy, ix <= 63 always
    }
}

__device__ __forceinline__ float conv1_win(const float (&xv)[9], const float* w1, float b1) {
  float v = b1;
#pragma unroll
  for (int k = 0; k < 9; k++) v = fmaf(w1[k], xv[k], v);
  return v;
}

// ---- 1. conv1 batch statistics from the input windows.  conv1 is linear in its
// 3x3 window x: v_c = b_c + w_c . x, so over the batch
//   E[v_c] = b_c + w_c . E[x],  E[v_c^2] = b_c^2 + 2 b_c w_c . E[x] + w_c' E[x x'] w_c
// and the 32 channels need only the 9 window means and 45 window products.
// One workgroup per 32 images; a thread owns 4 output positions (fp32 sums of
// 128 terms), the workgroup and grid sums are fp64.
constexpr int NMOM = 9 + 45;
constexpr int MOM_IMGS = 32;  // images per conv1_moments workgroup

__global__ __launch_bounds__(256) void conv1_moments_kernel(EncArgs a) {
  __shared__ __attribute__((aligned(16))) float x[IH][IW];
  __shared__ double red[4][NMOM];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  float m[NMOM];
#pragma unroll
  for (int k = 0; k < NMOM; k++) m[k] = 0.f;
  for (int i = 0; i < MOM_IMGS; i++) {
    const long long b = (long long)blockIdx.x * MOM_IMGS + i;
    if (b >= a.n) break;
    __syncthreads();
    stage_image(x, image_of(a, b));
    __syncthreads();
#pragma unroll
    for (int j = 0; j < H1 * H1 / 256; j++) {
      float xv[9];
      window(x, t + 256 * j, xv);
      int q = 9;
#pragma unroll
      for (int k = 0; k < 9; k++) {
        m[k] += xv[k];
#pragma unroll
        for (int l = k; l < 9; l++) m[q++] += xv[k] * xv[l];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NMOM; k++) {
    double d = m[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
    if (lane == 0) red[w][k] = d;
  }
  __syncthreads();
  if (t < NMOM) a.ws.part1[(long long)blockIdx.x * NMOM + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

// BN1 from the window moments (train mode): scale/shift and the running update
__global__ __launch_bounds__(256) void bn1_moments_kernel(EncArgs a, int nparts) {
  __shared__ double red[4][NMOM];
  __shared__ double mom[NMOM];
  const int t = threadIdx.x;
  if (t < 4 * NMOM) {
    const int k = t % NMOM, sub = t / NMOM;
    double s = 0.0;
    for (int p = sub; p < nparts; p += 4) s += a.ws.part1[(long long)p * NMOM + k];
    red[sub][k] = s;
  }
  __syncthreads();
  const double cnt = double(a.n) * (H1 * H1);
  if (t < NMOM) mom[t] = ((red[0][t] + red[1][t]) + (red[2][t] + red[3][t])) / cnt;
  __syncthreads();
  if (t >= C1) return;
  const int c = t;
  double wv[9];
  for (int k = 0; k < 9; k++) wv[k] = a.p.w1[c * 9 + k];
  const double b = a.p.b1[c];
  double wmu = 0.0, wMw = 0.0;
  int q = 9;
  for (int k = 0; k < 9; k++) {
    wmu += wv[k] * mom[k];
    for (int l = k; l < 9; l++) wMw += (k == l ? 1.0 : 2.0) * wv[k] * wv[l] * mom[q++];
  }
  const double mean = b + wmu;
  const double var = fmax(b * b + 2.0 * b * wmu + wMw - mean * mean, 0.0);
  a.p.rm1[c] = (1.f - a.momentum) * a.p.rm1[c] + a.momentum * float(mean);
  a.p.rv1[c] = (1.f - a.momentum) * a.p.rv1[c] + a.momentum * float(var * cnt / (cnt - 1.0));
  if (c == 0 && a.p.nbt1) *a.p.nbt1 += 1;
  const float sc = a.p.g1[c] / sqrtf(float(var) + a.eps);
  a.ws.ss1[c] = sc;
  a.ws.ss1[C1 + c] = a.p.be1[c] - float(mean) * sc;
}

// ---- 2. BN finish: batch (train) or running (eval) statistics -> scale/shift
// (and, in train mode, the running-statistics update torch's BatchNorm makes)
__global__ __launch_bounds__(256) void bn_finish_kernel(const double* part, int nparts, long long count, int C,
                                                        const float* gamma, const float* beta, float* rmean,
                                                        float* rvar, long long* nbt, int train, float momentum,
                                                        float eps, float* scale_shift) {
  __shared__ double red[8][32][2];
  const int c = threadIdx.x & 31, sub = threadIdx.x >> 5;  // C <= 32; 8 interleaved sub-sums
  if (train) {
    double s = 0.0, s2 = 0.0;
    if (c < C)
      for (int p = sub; p < nparts; p += 8) {
        s += part[((long long)p * C + c) * 2];
        s2 += part[((long long)p * C + c) * 2 + 1];
      }
    red[sub][c][0] = s;
    red[sub][c][1] = s2;
  }
  __syncthreads();
  if (sub != 0 || c >= C) return;
  float mean, var;
  if (train) {
    double s = 0.0, s2 = 0.0;
    for (int q = 0; q < 8; q++) { s += red[q][c][0]; s2 += red[q][c][1]; }
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

// ---- 3. conv2 as an implicit GEMM, producer/consumer.  One 512-thread
// workgroup per CU walks its images (grid-stride) in items of 8 input channels
// (4 items per image).  Waves 0-3 produce: conv1 + BN1 + LeakyReLU of item s's
// channels into LDS buffer s&1, each thread keeping its 4 positions' 3x3 input
// windows in registers for the whole image (read from global/L2, no LDS copy of
// the image).  Waves 4-7 consume item s-1 from buffer (s-1)&1 with MFMA: wave w
// owns position blocks 2w, 2w+1 (36 MFMA steps each per item).  A producer and a
// consumer wave share each SIMD, so the VALU work hides under the MFMAs.
constexpr int QCH = 8;  // conv1 channels per item

__global__ __launch_bounds__(512) void conv2_kernel(EncArgs a) {
  __shared__ float a1[2][QCH * CS];   // the activated conv1 output of one item, double-buffered
  __shared__ float w2t[K2][C1];       // conv2 weights, [ic*9 + tap][oc]
  __shared__ float ss1[2 * C1];
  __shared__ double red[4][C1][2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, hh = lane >> 5, oc = lane & 31;
  const bool producer = wv < 4;
  const int w = wv & 3, t8 = t & 255;
  for (int e = t; e < K2 * C1; e += 512) {
    const int o = e / K2, k = e % K2;
    w2t[k][o] = a.p.w2[e];
  }
  if (t < 2 * C1) ss1[t] = a.ws.ss1[t];
  __syncthreads();
  const float b2 = a.p.b2[oc];
  const long long nimg = a.n > blockIdx.x ? (a.n - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const long long nitems = 4 * nimg;
  double s = 0.0, s2 = 0.0;
  int py[2], px[2];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int pos = (2 * w + q) * 32 + (lane & 31);
    py[q] = pos >> 4;
    px[q] = pos & 15;
  }
  float xw[H1 * H1 / 256][9];  // producer: the input windows of its 4 positions
  f32x16 acc[2];
  for (long long st = 0; st <= nitems; st++) {
    if (producer && st < nitems) {
      const long long b = blockIdx.x + (st >> 2) * (long long)gridDim.x;
      const int quarter = int(st & 3), buf = int(st & 1);
      if (quarter == 0) {
        const float* img = image_of(a, b);
#pragma unroll
        for (int j = 0; j < H1 * H1 / 256; j++) {
          const int pos = t8 + 256 * j, oy = pos >> 5, ox = pos & 31;
#pragma unroll
          for (int ky = 0; ky < 3; ky++)
#pragma unroll
            for (int kx = 0; kx < 3; kx++) {
              const int iy = 2 * oy + ky - 1, ix = 2 * ox + kx - 1;
              xw[j][ky * 3 + kx] = (iy >= 0 && ix >= 0) ? img[iy * IW + ix] : 0.f;
            }
        }
      }
#pragma unroll
      for (int j = 0; j < H1 * H1 / 256; j++) {
        const int pos = t8 + 256 * j;
#pragma unroll
        for (int icl = 0; icl < QCH; icl++) {  // uniform channel: scalar weight loads
          const int ic = QCH * quarter + icl;
          a1[buf][icl * CS + pos] = leaky(fmaf(conv1_win(xw[j], a.p.w1 + ic * 9, a.p.b1[ic]), ss1[ic], ss1[C1 + ic]));
        }
      }
    }
    if (!producer && st >= 1) {
      const long long it = st - 1;
      const long long b = blockIdx.x + (it >> 2) * (long long)gridDim.x;
      const int quarter = int(it & 3), buf = int(it & 1);
      if (quarter == 0) {
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
          for (int r = 0; r < 16; r++) acc[q][r] = b2;
      }
      // K order: step (icp, tap): lane half hh takes input channel 2 icp + hh
#pragma unroll
      for (int icp = 0; icp < QCH / 2; icp++) {
        const int icl = 2 * icp + hh, ic = QCH * quarter + icl;
        const float* ach = a1[buf] + icl * CS;
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
      if (quarter == 3) {  // raw conv2 output, flattened (C, H, W): column = channel, rows = positions
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
    }
    __syncthreads();
  }
  if (a.train) {
    if (!producer) {
      s += __shfl_xor(s, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (hh == 0) { red[w][oc][0] = s; red[w][oc][1] = s2; }
    }
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
    const float v = ((tile[0][i][j] + tile[1][i][j]) + (tile[2][i][j] + tile[3][i][j])) + a.p.bl[j];
    tile[0][i][j] = im < a.n ? v : 0.f;
    if (im < a.n) a.ws.z[im * NZ + j] = v;
  }
  if (!a.train) return;
  __syncthreads();
  if (t < 2 * NZ) {  // this block's BatchNorm1d sums (fp64)
    const int j = t >> 1, k = t & 1;
    double sum = 0.0;
    for (int i = 0; i < 32; i++) {
      const double v = tile[0][i][j];
      sum += k ? v * v : v;
    }
    a.ws.part3[((long long)blockIdx.x * NZ + j) * 2 + k] = sum;
  }
}

// ---- 5. BatchNorm1d(20) + Tanh -> features.  Every workgroup forms the
// statistics from the linear kernel's per-block sums (same order, same bits);
// block 0 alone moves the running statistics.
__global__ __launch_bounds__(256) void head_kernel(EncArgs a, int nparts) {
  __shared__ double red[4][NZ][2];
  __shared__ float sc[NZ], sh[NZ];
  const int t = threadIdx.x;
  if (a.train) {
    if (t < 4 * 2 * NZ) {
      const int jk = t % (2 * NZ), sub = t / (2 * NZ);
      double s = 0.0;
      for (int p = sub; p < nparts; p += 4) s += a.ws.part3[(long long)p * 2 * NZ + jk];
      red[sub][jk >> 1][jk & 1] = s;
    }
    __syncthreads();
    if (t < NZ) {
      double S = 0.0, S2 = 0.0;
      for (int g = 0; g < 4; g++) { S += red[g][t][0]; S2 += red[g][t][1]; }
      const double cnt = double(a.n);
      const double m = S / cnt, v = fmax(S2 / cnt - m * m, 0.0);
      if (blockIdx.x == 0) {
        a.p.rm3[t] = (1.f - a.momentum) * a.p.rm3[t] + a.momentum * float(m);
        a.p.rv3[t] = (1.f - a.momentum) * a.p.rv3[t] + a.momentum * float(v * cnt / (cnt - 1.0));
        if (t == 0 && a.p.nbt3) *a.p.nbt3 += 1;
      }
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
  const long long e = (long long)blockIdx.x * 256 + t;
  if (e < a.n * NZ) {
    const int j = int(e % NZ);
    a.out[(e / NZ) * a.out_stride + j] = tanhf(fmaf(a.ws.z[e], sc[j], sh[j]));
  }
}

EncWorkspace carve(float* base, long long n, long long* total) {
  EncWorkspace w;
  long long o = 0;
  auto take = [&](long long nfloats) { float* p = base ? base + o : nullptr; o += (nfloats + 63) & ~63LL; return p; };
  const long long g1 = (n + 31) / 32;
  w.part1 = reinterpret_cast<double*>(take(g1 * NMOM * 2));
  w.part2 = reinterpret_cast<double*>(take(256LL * C1 * 2 * 2));
  w.ss1 = take(2 * C1);
  w.ss2 = take(2 * C1);
  w.out2 = take(n * FL);
  w.z = take(n * NZ);
  w.part3 = reinterpret_cast<double*>(take(((n + 31) / 32) * NZ * 2 * 2));
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
  const int g1 = int((a.n + MOM_IMGS - 1) / MOM_IMGS);
  const int g2 = int(a.n < 256 ? a.n : 256);
  if (a.train) {
    hipLaunchKernelGGL(conv1_moments_kernel, dim3(g1), dim3(256), 0, s, a);
    hipLaunchKernelGGL(bn1_moments_kernel, dim3(1), dim3(256), 0, s, a, g1);
  } else {
    hipLaunchKernelGGL(bn_finish_kernel, dim3(1), dim3(256), 0, s, (const double*)a.ws.part1, g1, a.n * H1 * H1, C1,
                       a.p.g1, a.p.be1, a.p.rm1, a.p.rv1, a.p.nbt1, 0, a.momentum, a.eps, a.ws.ss1);
  }
  hipLaunchKernelGGL(conv2_kernel, dim3(g2), dim3(512), 0, s, a);
  hipLaunchKernelGGL(bn_finish_kernel, dim3(1), dim3(256), 0, s, (const double*)a.ws.part2, g2, a.n * H2 * H2, C1,
                     a.p.g2, a.p.be2, a.p.rm2, a.p.rv2, a.p.nbt2, a.train, a.momentum, a.eps, a.ws.ss2);
  hipLaunchKernelGGL(linear_kernel, dim3(int((a.n + 31) / 32)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(head_kernel, dim3(int((a.n * NZ + 255) / 256)), dim3(256), 0, s, a, int((a.n + 31) / 32));
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
