// bb_encoder.h -- the fused frozen depth encoder (bb_encoder.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

struct EncParams {
  const float *w1, *b1, *g1, *be1;  // conv1 [32][1][3][3], [32]; BatchNorm2d weight, bias
  float *rm1, *rv1;                 // running mean / var (updated in train mode)
  long long* nbt1;                  // num_batches_tracked (may be NULL)
  const float *w2, *b2, *g2, *be2;  // conv2 [32][32][3][3], [32]; BatchNorm2d
  float *rm2, *rv2;
  long long* nbt2;
  const float *wl, *bl, *g3, *be3;  // Linear [20][8192], [20]; BatchNorm1d
  float *rm3, *rv3;
  long long* nbt3;
};

struct EncWorkspace {
  double* part1;  // conv1 input-window moments per workgroup
  double* part2;  // conv2 channel sums per workgroup
  float* ss1;     // BN1 scale, shift
  float* ss2;     // BN2 scale, shift
  float* out2;    // [n][8192] raw conv2 output
  float* z;       // [n][20] raw linear output
  double* part3;  // BatchNorm1d sums per 32-image block
};

struct EncArgs {
  EncParams p;
  const float* images;     // image i at images + i * image_stride, 64x64 row-major
  long long image_stride;  // floats
  const long long* index;  // NULL, or image i is row index[i] of images (a minibatch gather)
  long long n;
  int train;
  float momentum, eps;
  float* out;              // features: row i at out + i * out_stride
  long long out_stride;
  EncWorkspace ws;
};

long long encoder_workspace_bytes(long long n);
int launch_encoder(EncArgs a, float* ws, hipStream_t s);

}  // namespace bb
