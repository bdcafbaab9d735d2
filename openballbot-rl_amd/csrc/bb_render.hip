// bb_render.hip -- robot-mounted depth cameras.
//
// The reference renders cam_0 / cam_1 (ballbot.xml:44-54, fovy 90, 64x64,
// depth only) through MuJoCo's OpenGL renderer every ceil((1/90 s)/2 ms) = 6
// physics steps (ballbot_env.py:389-411, 743-767) and clips depth at 1 m
// (sensors/rgbd.py:46-82).  Here every (env, camera) is one workgroup that
// ray-casts its image: the linear eye-space depth of the nearest front face
// among the hfield surface, the ball, the tower cylinder, the cam sticks and
// the wheel capsules, clipped to 1.  The geometry and conventions are those of
// oracle/bb_oracle.c:bbo_render_depth (fp64), the checker of this kernel.
//
// Work: scene_kernel (one thread per env) runs the fixed-tree kinematics
// (bb_physics.h) and writes both cameras' frames and the 7 primitives (220 B
// per camera); depth_kernel stages one scene in LDS and its 256 threads cast
// H*W rays (16 each at 64x64).  Rays stop at z-depth 1 m, so the hfield
// DDA visits at most ~100 cells (cell 34 mm, ray <= sqrt(3) m); a typical ray
// hits the ground within ~10.  Only envs whose step counter is a multiple of
// the frame interval render (the others keep their last image), so on average
// 1/6 of the workgroups do work.  Output: depth f32[n][2][H][W] (obs rgbd_0 =
// [:, 0:1], rgbd_1 = [:, 1:2]) and relative_image_timestamp f32[n].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_physics.h"
#include "bb_render.h"

namespace bb {
namespace {

constexpr float ZNEAR = 1e-4f * 14.142135623730951f;  // ballbot.xml:8 znear * extent

struct Scene {
  float o[3], R[9];     // camera origin, camera->world rotation (columns: x right, y up, z back)
  float ball[3];
  float pa[6][3], pb[6][3];  // 0 tower (cylinder), 1-2 sticks, 3-5 wheels (capsules)
  float rad[6];
  float size_z;
  float ztop;  // max terrain height (hmax * size_z): rays above it skip the march
  int tid;
};

__device__ __forceinline__ float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__device__ float ray_sphere(const float* o, const float* d, const float* c, float r) {
  const float oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
  const float b = dot3(oc, d), cc = dot3(oc, oc) - r * r, h = b * b - cc;
  return h < 0.f ? -1.f : -b - sqrtf(h);
}

__device__ float ray_capsule(const float* o, const float* d, const float* pa, const float* pb, float r) {
  const float ba[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  const float oa[3] = {o[0] - pa[0], o[1] - pa[1], o[2] - pa[2]};
  const float baba = dot3(ba, ba), bard = dot3(ba, d), baoa = dot3(ba, oa), rdoa = dot3(d, oa), oaoa = dot3(oa, oa);
  const float a = baba - bard * bard, b = baba * rdoa - baoa * bard, c = baba * oaoa - baoa * baoa - r * r * baba;
  const float h = b * b - a * c;
  if (h < 0.f) return -1.f;
  const bool body = a > 1e-30f;
  const float t = body ? (-b - sqrtf(h)) / a : -1.f;
  const float y = baoa + t * bard;
  if (body && y > 0.f && y < baba) return t;
  float oc[3];
  if (y <= 0.f) { oc[0] = oa[0]; oc[1] = oa[1]; oc[2] = oa[2]; }
  else { oc[0] = o[0] - pb[0]; oc[1] = o[1] - pb[1]; oc[2] = o[2] - pb[2]; }
  const float bb = dot3(d, oc), cc = dot3(oc, oc) - r * r, hh = bb * bb - cc;
  return hh > 0.f ? -bb - sqrtf(hh) : -1.f;
}

__device__ float ray_cylinder(const float* o, const float* d, const float* pa, const float* pb, float r) {
  const float ba[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  const float oc[3] = {o[0] - pa[0], o[1] - pa[1], o[2] - pa[2]};
  const float baba = dot3(ba, ba), bard = dot3(ba, d), baoc = dot3(ba, oc);
  const float k2 = baba - bard * bard, k1 = baba * dot3(oc, d) - baoc * bard;
  const float k0 = baba * dot3(oc, oc) - baoc * baoc - r * r * baba;
  float h = k1 * k1 - k2 * k0;
  if (h < 0.f) return -1.f;
  h = sqrtf(h);
  if (k2 > 1e-30f) {
    float t = (-k1 - h) / k2;
    const float y = baoc + t * bard;
    if (y > 0.f && y < baba) return t;
    if (fabsf(bard) < 1e-30f) return -1.f;
    t = (((y < 0.f) ? 0.f : baba) - baoc) / bard;
    return fabsf(k1 + k2 * t) < h ? t : -1.f;
  }
  if (k0 > 0.f || fabsf(bard) < 1e-30f) return -1.f;
  const float t0 = -baoc / bard, t1 = (baba - baoc) / bard;
  return fminf(t0, t1);
}

__device__ float ray_tri(const float* o, const float* d, const float* a, const float* b, const float* c) {
  const float e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  const float p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
  const float det = dot3(e1, p);
  if (fabsf(det) < 1e-30f) return -1.f;
  const float inv = 1.f / det;
  const float s[3] = {o[0] - a[0], o[1] - a[1], o[2] - a[2]};
  const float u = dot3(s, p) * inv;
  if (u < 0.f || u > 1.f) return -1.f;
  const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
  const float v = dot3(d, q) * inv;
  if (v < 0.f || u + v > 1.f) return -1.f;
  return dot3(e2, q) * inv;
}

// nearest hfield hit in (tmin, tmax) by a 2-D DDA over the cells the ray crosses
__device__ float ray_hfield(const float* o, const float* d, const float* hf, float size_z, float ztop, float sx,
                            float sy, float tmin, float tmax) {
  const int N1 = HF_N - 1;
  const float dx = 2.f * sx / N1, dy = 2.f * sy / N1;
  float t0 = tmin, t1 = tmax;
  // no surface above ztop: start where the ray descends through it (flat: the plane hit)
  if (o[2] > ztop) {
    if (d[2] >= 0.f) return -1.f;
    t0 = fmaxf(t0, (ztop - o[2]) / d[2] * (1.f - 1e-6f));
  }
  const float half[2] = {sx, sy};
#pragma unroll
  for (int ax = 0; ax < 2; ax++) {
    if (fabsf(d[ax]) < 1e-30f) {
      if (o[ax] < -half[ax] || o[ax] > half[ax]) return -1.f;
      continue;
    }
    float ta = (-half[ax] - o[ax]) / d[ax], tb = (half[ax] - o[ax]) / d[ax];
    if (ta > tb) { const float s = ta; ta = tb; tb = s; }
    t0 = fmaxf(t0, ta);
    t1 = fminf(t1, tb);
  }
  const float px = o[0] + t0 * d[0], py = o[1] + t0 * d[1];
  // negated: a NaN camera pose (diverged state) casts no ray into the field
  if (!(t0 <= t1) || !(fabsf(px) <= 2.f * sx && fabsf(py) <= 2.f * sy)) return -1.f;
  int c = (int)floorf((px + sx) / dx), r = (int)floorf((py + sy) / dy);
  c = c < 0 ? 0 : (c > N1 - 1 ? N1 - 1 : c);
  r = r < 0 ? 0 : (r > N1 - 1 ? N1 - 1 : r);
  const int stc = d[0] > 0.f ? 1 : -1, str = d[1] > 0.f ? 1 : -1;
  const float tdx = fabsf(d[0]) > 1e-30f ? dx / fabsf(d[0]) : 1e30f;
  const float tdy = fabsf(d[1]) > 1e-30f ? dy / fabsf(d[1]) : 1e30f;
  float tmx = fabsf(d[0]) > 1e-30f ? (-sx + (c + (stc > 0)) * dx - o[0]) / d[0] : 1e30f;
  float tmy = fabsf(d[1]) > 1e-30f ? (-sy + (r + (str > 0)) * dy - o[1]) / d[1] : 1e30f;
  for (int it = 0; it < 4 * HF_N; it++) {
    const float x0 = -sx + c * dx, x1 = -sx + (c + 1) * dx, y0 = -sy + r * dy, y1 = -sy + (r + 1) * dy;
    const float A[3] = {x0, y0, hf[r * HF_N + c] * size_z}, B[3] = {x0, y1, hf[(r + 1) * HF_N + c] * size_z};
    const float C[3] = {x1, y0, hf[r * HF_N + c + 1] * size_z}, D[3] = {x1, y1, hf[(r + 1) * HF_N + c + 1] * size_z};
    float best = -1.f;
    const float ta = ray_tri(o, d, A, B, C), tb = ray_tri(o, d, B, C, D);
    if (ta > tmin && ta < tmax) best = ta;
    if (tb > tmin && tb < tmax && (best < 0.f || tb < best)) best = tb;
    if (best > 0.f) return best;
    if (fminf(tmx, tmy) > t1) break;
    if (tmx < tmy) {
      c += stc; tmx += tdx;
      if (c < 0 || c > N1 - 1) break;
    } else {
      r += str; tmy += tdy;
      if (r < 0 || r > N1 - 1) break;
    }
  }
  return -1.f;
}

__device__ void to_world(const Kin<float>& k, const float* pl, float* pw) {
  float t[3];
  mv3(t, k.Rb, pl);
  pw[0] = k.pb[0] + t[0]; pw[1] = k.pb[1] + t[1]; pw[2] = k.pb[2] + t[2];
}

// one thread per env: camera frames and primitives of both cameras -> scenes[e][cam]
template <typename T>
__global__ __launch_bounds__(64) void scene_kernel(ModelT<float> m, CamRig rig, RenderDev d, int every, int force,
                                                   float dt, Scene* __restrict__ scenes, float* __restrict__ rel_ts) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.n) return;
  const int k6 = d.steps[e] % every;
  if (rel_ts) rel_ts[e] = float(double(k6) * double(dt));
  if (!force && k6 != 0) return;
  const T* Q = (const T*)d.qpos;
  float q[NQ];
#pragma unroll
  for (int i = 0; i < NQ; i++) q[i] = float(Q[size_t(i) * d.n + e]);
  Kin<float> k;
  kinematics(m, q, k);
  Scene S;
  S.ball[0] = k.c[0]; S.ball[1] = k.c[1]; S.ball[2] = k.c[2];
  float a[3], p[3];
  for (int s = -1; s <= 1; s += 2) {  // tower cylinder along the base z axis
    p[0] = m.tower_c[0]; p[1] = m.tower_c[1]; p[2] = m.tower_c[2] + s * m.tower_hh;
    to_world(k, p, s < 0 ? S.pa[0] : S.pb[0]);
  }
  S.rad[0] = m.tower_r;
  for (int c = 0; c < 2; c++) {
    for (int s = -1; s <= 1; s += 2) {
      for (int i = 0; i < 3; i++) p[i] = m.stick_c[c][i] + s * m.stick_hh * m.stick_a[c][i];
      to_world(k, p, s < 0 ? S.pa[1 + c] : S.pb[1 + c]);
    }
    S.rad[1 + c] = m.stick_r;
  }
  for (int w = 0; w < 3; w++) {
    mv3(a, k.Rw[w], m.gz);
    for (int s = -1; s <= 1; s += 2) {
      for (int i = 0; i < 3; i++) p[i] = k.wc[w][i] + s * m.wheel_hh * a[i];
      to_world(k, p, s < 0 ? S.pa[3 + w] : S.pb[3 + w]);
    }
    S.rad[3 + w] = m.wheel_r;
  }
  S.tid = d.terrain[e];
  S.size_z = d.size_z[S.tid];
  S.ztop = d.hmax[S.tid] * S.size_z;
  for (int cam = 0; cam < 2; cam++) {
    to_world(k, rig.p[cam], S.o);
    mm3(S.R, k.Rb, rig.R[cam]);
    scenes[2 * e + cam] = S;
  }
}

// one workgroup per (env, camera): H*W rays against the scene
__global__ __launch_bounds__(256) void depth_kernel(ModelT<float> m, RenderDev d, const Scene* __restrict__ scenes,
                                                    int H, int W, int every, int force, float* __restrict__ depth) {
  const int e = blockIdx.x >> 1, cam = blockIdx.x & 1;
  if (e >= d.n) return;
  if (!force && d.steps[e] % every != 0) return;
  __shared__ Scene S;
  constexpr int NW = sizeof(Scene) / sizeof(float);
  static_assert(sizeof(Scene) % sizeof(float) == 0, "Scene is copied as floats");
  if (threadIdx.x < NW)
    reinterpret_cast<float*>(&S)[threadIdx.x] = reinterpret_cast<const float*>(scenes + 2 * e + cam)[threadIdx.x];
  __syncthreads();
  const float* hf = d.bank + size_t(S.tid) * (HF_N * HF_N);
  float* out = depth + (size_t(e) * 2 + cam) * H * W;
  const float aspect = float(W) / float(H);
  for (int px = threadIdx.x; px < H * W; px += blockDim.x) {
    const int i = px / W, j = px - i * W;
    const float xc = (2.f * (j + 0.5f) / W - 1.f) * aspect, yc = 1.f - 2.f * (i + 0.5f) / H;  // tan(fovy/2) = 1
    float dr[3] = {S.R[0] * xc + S.R[1] * yc - S.R[2], S.R[3] * xc + S.R[4] * yc - S.R[5],
                   S.R[6] * xc + S.R[7] * yc - S.R[8]};
    const float len = sqrtf(dot3(dr, dr)), il = 1.f / len;
    dr[0] *= il; dr[1] *= il; dr[2] *= il;
    const float tmin = ZNEAR * len;
    float best = len;  // z-depth 1
    const float tb = ray_sphere(S.o, dr, S.ball, m.ball_r);
    if (tb > tmin && tb < best) best = tb;
    {
      const float t = ray_cylinder(S.o, dr, S.pa[0], S.pb[0], S.rad[0]);
      if (t > tmin && t < best) best = t;
    }
#pragma unroll 1
    for (int g = 1; g < 6; g++) {
      const float t = ray_capsule(S.o, dr, S.pa[g], S.pb[g], S.rad[g]);
      if (t > tmin && t < best) best = t;
    }
    const float tg = ray_hfield(S.o, dr, hf, S.size_z, S.ztop, m.hf_sx, m.hf_sy, tmin, best);
    if (tg > tmin && tg < best) best = tg;
    out[px] = fminf(best * il, 1.f);
  }
}

}  // namespace

size_t scene_bytes(int n) { return sizeof(Scene) * 2 * size_t(n); }

int launch_depth(bool fp64, const ModelT<float>& m, const CamRig& rig, const RenderDev& d, int H, int W, int every,
                 int force, float dt, void* scenes, float* depth, float* rel_ts, hipStream_t s) {
  if (d.n <= 0) return 0;
  Scene* sc = (Scene*)scenes;
  if (fp64)
    hipLaunchKernelGGL(scene_kernel<double>, dim3((d.n + 63) / 64), dim3(64), 0, s, m, rig, d, every, force, dt, sc,
                       rel_ts);
  else
    hipLaunchKernelGGL(scene_kernel<float>, dim3((d.n + 63) / 64), dim3(64), 0, s, m, rig, d, every, force, dt, sc,
                       rel_ts);
  hipLaunchKernelGGL(depth_kernel, dim3(2 * d.n), dim3(256), 0, s, m, d, sc, H, W, every, force, depth);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace bb
