// bb_terrain.hip -- terrain bank generation on the GPU.
//
// The reference regenerates a perlin heightfield at every reset with 85,849
// Python-level noise.snoise2 calls (terrain/perlin.py:49-68, ballbot_env.py:
// 501-513); that loop dominates its perlin throughput.  Here the whole seed
// space the reset draws from (integers(0, 10000), ballbot_env.py:505-510) is
// generated once, in one launch, into the device terrain bank, so a reset only
// picks a terrain id.
//
// Algorithm: snoise2(x, y, octaves, persistence, lacunarity, repeatx=repeaty=
// 1024, base=seed) of caseman/noise 1.2.x (not vendored; its published
// algorithm is restated in ballbot_gym/terrain/perlin.py, the checker of this
// kernel): the tiled 2-D noise is 4-D simplex fBm on a torus built with the
// library's polynomial fast_sin/fast_cos.  Every float operation is written in
// the order of that restatement with FMA contraction off, so the bank is
// bit-identical to the numpy restatement (tests/test_gpu_parity.py).
//
// Layout: bank float[n_terrains][293*293] row-major (row i <-> y, column j <->
// x in MuJoCo); one thread per vertex, grid.y = terrain.  HBM-write bound:
// 343 KB per terrain, a 10^4-seed bank is 3.4 GB.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_terrain.h"

namespace bb {
namespace {

__constant__ unsigned char PERM[512] = {
    151, 160, 137, 91,  90,  15,  131, 13,  201, 95,  96,  53,  194, 233, 7,   225, 140, 36,  103, 30,  69,  142,
    8,   99,  37,  240, 21,  10,  23,  190, 6,   148, 247, 120, 234, 75,  0,   26,  197, 62,  94,  252, 219, 203,
    117, 35,  11,  32,  57,  177, 33,  88,  237, 149, 56,  87,  174, 20,  125, 136, 171, 168, 68,  175, 74,  165,
    71,  134, 139, 48,  27,  166, 77,  146, 158, 231, 83,  111, 229, 122, 60,  211, 133, 230, 220, 105, 92,  41,
    55,  46,  245, 40,  244, 102, 143, 54,  65,  25,  63,  161, 1,   216, 80,  73,  209, 76,  132, 187, 208, 89,
    18,  169, 200, 196, 135, 130, 116, 188, 159, 86,  164, 100, 109, 198, 173, 186, 3,   64,  52,  217, 226, 250,
    124, 123, 5,   202, 38,  147, 118, 126, 255, 82,  85,  212, 207, 206, 59,  227, 47,  16,  58,  17,  182, 189,
    28,  42,  223, 183, 170, 213, 119, 248, 152, 2,   44,  154, 163, 70,  221, 153, 101, 155, 167, 43,  172, 9,
    129, 22,  39,  253, 19,  98,  108, 110, 79,  113, 224, 232, 178, 185, 112, 104, 218, 246, 97,  228, 251, 34,
    242, 193, 238, 210, 144, 12,  191, 179, 162, 241, 81,  51,  145, 235, 249, 14,  239, 107, 49,  192, 214, 31,
    181, 199, 106, 157, 184, 84,  204, 176, 115, 121, 50,  45,  127, 4,   150, 254, 138, 236, 205, 93,  222, 114,
    67,  29,  24,  72,  243, 141, 128, 195, 78,  66,  215, 61,  156, 180,
    151, 160, 137, 91,  90,  15,  131, 13,  201, 95,  96,  53,  194, 233, 7,   225, 140, 36,  103, 30,  69,  142,
    8,   99,  37,  240, 21,  10,  23,  190, 6,   148, 247, 120, 234, 75,  0,   26,  197, 62,  94,  252, 219, 203,
    117, 35,  11,  32,  57,  177, 33,  88,  237, 149, 56,  87,  174, 20,  125, 136, 171, 168, 68,  175, 74,  165,
    71,  134, 139, 48,  27,  166, 77,  146, 158, 231, 83,  111, 229, 122, 60,  211, 133, 230, 220, 105, 92,  41,
    55,  46,  245, 40,  244, 102, 143, 54,  65,  25,  63,  161, 1,   216, 80,  73,  209, 76,  132, 187, 208, 89,
    18,  169, 200, 196, 135, 130, 116, 188, 159, 86,  164, 100, 109, 198, 173, 186, 3,   64,  52,  217, 226, 250,
    124, 123, 5,   202, 38,  147, 118, 126, 255, 82,  85,  212, 207, 206, 59,  227, 47,  16,  58,  17,  182, 189,
    28,  42,  223, 183, 170, 213, 119, 248, 152, 2,   44,  154, 163, 70,  221, 153, 101, 155, 167, 43,  172, 9,
    129, 22,  39,  253, 19,  98,  108, 110, 79,  113, 224, 232, 178, 185, 112, 104, 218, 246, 97,  228, 251, 34,
    242, 193, 238, 210, 144, 12,  191, 179, 162, 241, 81,  51,  145, 235, 249, 14,  239, 107, 49,  192, 214, 31,
    181, 199, 106, 157, 184, 84,  204, 176, 115, 121, 50,  45,  127, 4,   150, 254, 138, 236, 205, 93,  222, 114,
    67,  29,  24,  72,  243, 141, 128, 195, 78,  66,  215, 61,  156, 180};

// 4-D gradient gi (0..31): the edge midpoints of the 4-cube, component
// (gi >> 3) zero, the other three +-1 with signs from bits 2,1,0 of gi (set =
// negative) -- the order of the restatement's GRAD4 table.
__device__ __forceinline__ float grad4_dot(int gi, float x, float y, float z, float w) {
#pragma clang fp contract(off)
  const int zero = gi >> 3;
  const float s0 = (gi & 4) ? -1.f : 1.f, s1 = (gi & 2) ? -1.f : 1.f, s2 = (gi & 1) ? -1.f : 1.f;
  float g[4];
  int k = 0;
  const float sg[3] = {s0, s1, s2};
#pragma unroll
  for (int c = 0; c < 4; c++) g[c] = (c == zero) ? 0.f : sg[k++];
  return g[0] * x + g[1] * y + g[2] * z + g[3] * w;
}

// caseman/noise _noise.h fast_sin: x in [0, 2] <-> angle [0, 2 pi]
__device__ __forceinline__ float fast_sin(float x) {
#pragma clang fp contract(off)
  const float z = x + 25165824.0f;
  x = x - (z - 25165824.0f);
  const float y = x - x * fabsf(x);
  return y * (3.1f + 3.6f * fabsf(y));
}

__device__ float noise4(float x, float y, float z, float w) {
#pragma clang fp contract(off)
  const float F4 = 0.30901699437494745f, G4 = 0.1381966011250105f;  // (sqrt5-1)/4, (5-sqrt5)/20
  const float s = (x + y + z + w) * F4;
  const float i = floorf(x + s), j = floorf(y + s), k = floorf(z + s), l = floorf(w + s);
  const float t = (i + j + k + l) * G4;
  const float x0 = x - (i - t), y0 = y - (j - t), z0 = z - (k - t), w0 = w - (l - t);
  // simplex corner order by coordinate rank (ties as the reference's table)
  const int rx = (x0 > y0) + (x0 > z0) + (x0 > w0);
  const int ry = (y0 >= x0) + (y0 > z0) + (y0 > w0);
  const int rz = (z0 >= x0) + (z0 >= y0) + (z0 > w0);
  const int rw = (w0 >= x0) + (w0 >= y0) + (w0 >= z0);
  const int I = int(i) & 255, J = int(j) & 255, K = int(k) & 255, L = int(l) & 255;
  float total = 0.f;
#pragma unroll
  for (int c = 0; c < 5; c++) {
    // corner c: offsets o = rank >= 4-c (c=0: none, c=4: all)
    const int th = 4 - c;
    const int ox = rx >= th, oy = ry >= th, oz = rz >= th, ow = rw >= th;
    const float gc = float(c) * G4;
    float px, py, pz, pw;
    if (c == 0) { px = x0; py = y0; pz = z0; pw = w0; }
    else if (c == 4) { px = x0 - 1.f + 4.f * G4; py = y0 - 1.f + 4.f * G4; pz = z0 - 1.f + 4.f * G4; pw = w0 - 1.f + 4.f * G4; }
    else { px = x0 - float(ox) + gc; py = y0 - float(oy) + gc; pz = z0 - float(oz) + gc; pw = w0 - float(ow) + gc; }
    const float f = 0.6f - px * px - py * py - pz * pz - pw * pw;
    const int gi = PERM[I + ox + PERM[J + oy + PERM[K + oz + PERM[L + ow]]]] & 0x1F;
    const float dot = grad4_dot(gi, px, py, pz, pw);
    total = total + (f > 0.f ? (f * f) * (f * f) * dot : 0.f);
  }
  return total * 27.0f;
}

__global__ __launch_bounds__(256) void perlin_kernel(float* __restrict__ bank, const int32_t* __restrict__ seeds,
                                                     PerlinCfg cfg) {
#pragma clang fp contract(off)
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= HF_VERTS) return;
  const int t = blockIdx.y;
  const int i = v / HF_N_, j = v - i * HF_N_;
  // snoise2(i/scale, j/scale, ..., repeatx=repeaty=R, base=seed)
  const float xin = float(double(i) / cfg.scale), yin = float(double(j) / cfg.scale);
  const float base = float(seeds[t]);
  const float R = 1024.0f;
  const float rr = float(double(R) * 0.31830988618379067154 * 0.5);  // R / (2 pi)
  const float yf = float(double(yin) * 2.0 / double(R));
  const float xf = float(double(xin) * 2.0 / double(R));
  const float y4 = fast_sin(yf) * rr, w4 = base + fast_sin(yf + 0.5f) * rr;
  const float x4 = fast_sin(xf) * rr, z4 = base + fast_sin(xf + 0.5f) * rr;
  float total = noise4(x4, y4, z4, w4);
  float amp = 1.f, freq = 1.f, mx = 1.f;
  for (int o = 1; o < cfg.octaves; o++) {
    freq = freq * cfg.lacunarity;
    amp = amp * cfg.persistence;
    mx = mx + amp;
    total = total + noise4(x4 * freq, y4 * freq, z4 * freq, w4 * freq) * amp;
  }
  const float nv = float(double(total) / double(mx));  // correctly rounded float division
  double h = (double(nv) + 1.0) / 2.0 * cfg.amplitude;
  h = h < 0.0 ? 0.0 : (h > 1.0 ? 1.0 : h);
  bank[size_t(t) * HF_VERTS + v] = float(h);
}

// per terrain: init offset (ballbot_env.py:546-563: window max * size_z + 0.01
// with the reference's cell = size/nrows, i.e. rows/cols [140, 152)) and the
// global max height (the kernels' base-tree contact pre-filter)
__global__ __launch_bounds__(256) void terrain_stats_kernel(const float* __restrict__ bank, float size_z,
                                                            float* __restrict__ offset, float* __restrict__ hmax) {
  __shared__ float red[2][256];
  const int t = blockIdx.x;
  const float* hf = bank + size_t(t) * HF_VERTS;
  float gm = 0.f, wm = -3.0e38f;
  for (int v = threadIdx.x; v < HF_VERTS; v += blockDim.x) {
    const float x = hf[v];
    gm = fmaxf(gm, x);
    const int r = v / HF_N_, c = v - r * HF_N_;
    if (r >= HF_WIN0 && r < HF_WIN1 && c >= HF_WIN0 && c < HF_WIN1) wm = fmaxf(wm, x);
  }
  red[0][threadIdx.x] = gm;
  red[1][threadIdx.x] = wm;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] = fmaxf(red[0][threadIdx.x], red[0][threadIdx.x + s]);
      red[1][threadIdx.x] = fmaxf(red[1][threadIdx.x], red[1][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    hmax[t] = red[0][0];
    offset[t] = float(double(red[1][0]) * double(size_z) + 0.01);
  }
}

}  // namespace

int launch_perlin_bank(float* bank, const int32_t* seeds_dev, int count, const PerlinCfg& cfg, float size_z,
                       float* offset, float* hmax, hipStream_t s) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(perlin_kernel, dim3((HF_VERTS + 255) / 256, count), dim3(256), 0, s, bank, seeds_dev, cfg);
  hipLaunchKernelGGL(terrain_stats_kernel, dim3(count), dim3(256), 0, s, bank, size_z, offset, hmax);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
