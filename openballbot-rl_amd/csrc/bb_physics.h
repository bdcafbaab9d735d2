// bb_physics.h -- specialised per-env ballbot physics (one env per lane).
//
// MI355X-native re-derivation of the reference hot path
// `mujoco.mj_step(model, data)` (ballbot_gym/envs/ballbot_env.py:912) for the
// one fixed model ballbot_gym/models/ballbot.xml, plus the step glue of
// BBotSimulation.step (ballbot_env.py:854-1036).  It is NOT a port of MuJoCo:
// every quantity is derived in closed form for this tree
//   world -> base(free) -> {cam_0, cam_1 (welded, merged), wheel_0..2 (hinge)}
//   world -> ball(free)
// * mass matrix: constant local-frame blocks + 3 hinge columns (build_mass)
// * bias forces: two-level spatial RNE in body-local coordinates (bias_forces)
// * contacts: patched sphere-capsule pairs (tools/mujoco_fix.patch) and the
//   exact sphere / hfield-prism penetration (collide_ground)
// * elliptic-cone Newton solve on a register-resident packed 15x15 Hessian
//   with exact line search (solve)
// * RK4 (mj_RungeKutta N=4) with quaternion integration (rk4_step)
// Ball-terrain contacts (dynamic count, <= MAXG) live in a per-lane store
// (LDS, lane-interleaved, on the GPU).
//
// Templated on the arithmetic type T (float or double); compiled for gfx950
// (bb_kernels.hip) and, for tests only, for the host (tests/hostcheck).
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define BB_HD __host__ __device__ __forceinline__

namespace bb {

constexpr int NQ = 17, NV = 15, NU = 3;
constexpr int HF_N = 293;        // ballbot.xml:23 nrow = ncol
constexpr int MAXG = 50;         // ball-hfield contact cap: MuJoCo's mjMAXCONPAIR (== oracle BBO_MAXGROUND)
constexpr int NH = NV * (NV + 1) / 2;
constexpr int NGF = 4;           // fields per stored ground contact (see GF_* below)
constexpr int MAXPAIR = 50;      // contacts per hfield x geom pair: MuJoCo's mjMAXCONPAIR (== oracle BBO_MAXPAIR)
constexpr int MAXB = 3 + 6 * MAXPAIR;  // base-tree geom contacts (== oracle BBO_MAXBODY)
constexpr int MAXB_LDS = 32;     // of which in the team's LDS; the rest spill to a per-env HBM block
constexpr int NBF = 8;           // fields per stored base-tree contact (see BF_* below)
// ground-contact store fields (compact: Jacobian, aref and D are rebuilt on
// use by ground_contact): normal (hfield -> ball)[3], dist
constexpr int GF_N = 0, GF_DIST = 3;
// base-tree contact store: normal (geom1 -> geom2)[3], position (world)[3],
// dist, body code 8*body1 + body2 (body1: 0 world / 7 ball; body2: 1 base,
// 2-3 cam bodies, 4-6 wheels)
constexpr int BF_N = 0, BF_P = 3, BF_DIST = 6, BF_CODE = 7;

// ------------------------------------------------------------------ model
// Compiled constants (bb_model.cpp computes them in double from the MJCF
// table, then uses this file's own mass matrix for invweight0).
template <typename T>
struct ModelT {
  // base tree rigid part = base + cam_0_body + cam_1_body (welded), base-local
  T m0, h0[3], I0O[6];   // mass, first moment, inertia about base origin (xx,yy,zz,xy,xz,yz)
  // wheel bodies (identical), wheel-body frame
  T mw, cw[3], Iw[6];    // mass, COM (= capsule centre), inertia about COM
  T gz[3];               // capsule axis in wheel frame
  T wq[3][4];            // wheel body quat in base frame (euler 0,0,120k; ballbot.xml:56,61,67)
  T axis[3];             // hinge axis in wheel frame (normalised; ballbot.xml:58)
  T u[3][3];             // hinge axis in base frame
  T jpos[3];             // hinge anchor in wheel frame
  T anchor[3];           // hinge anchor in base frame
  T wheel_r, wheel_hh, armature, damping;
  // ball
  T mB, IB, ball_r, dz;  // geom offset (0,0,dz) in ball frame (ballbot.xml:78)
  // base-tree collision geoms (dynamic pairs), base frame
  T tower_c[3], tower_r, tower_hh;         // cylinder (ballbot.xml:41), axis = base z
  T stick_c[2][3], stick_a[2][3], stick_r, stick_hh;  // cam sticks (capsules, ballbot.xml:46,52)
  // constraint parameters
  T iw_ball, iw_wheel[3];  // body_invweight0 (translational)
  T iw_base, iw_cam[2];
  T K, Bd;                 // solref (0.02,1) -> stiffness, damping
  T solimp[5];             // (0.9, 0.95, 0.001, 0.5, 2)
  T fr_wheel[2];           // pair friction (0.001, 1.0) (ballbot.xml:90-92)
  // options / solver
  T h, grav;
  T hf_sx, hf_sy, hf_bottom;
  T scale, tol, ls_tol, step_rel2;  // step_rel2: stop when |alpha s|^2 <= step_rel2 (1 + |a|^2)
  int maxiter, ls_maxiter;
  T qpos0[NQ];
};

// ------------------------------------------------------------- helpers
template <typename T> BB_HD T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename T> BB_HD void cross3(T* r, const T* a, const T* b) {
  T x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}
// x[6 + w] for a runtime w in {0,1,2}, without an indexed load: LLVM folds
// `w == 0 ? x[6] : ...` into x[6 + w], which turns the whole register array x
// into a scratch-memory array.  Bit masks keep it a register select.
template <typename T>
BB_HD T hinge_sel(int w, const T* x) {
  using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned int>::type;
  const U m0 = U(0) - U(w == 0), m1 = U(0) - U(w == 1), m2 = U(0) - U(w == 2);
  const U b = (__builtin_bit_cast(U, x[6]) & m0) | (__builtin_bit_cast(U, x[7]) & m1) | (__builtin_bit_cast(U, x[8]) & m2);
  return __builtin_bit_cast(T, b);
}

template <typename T> BB_HD void mv3(T* r, const T* M, const T* v) {  // r = M v
  T x = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  T y = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  T z = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  r[0] = x; r[1] = y; r[2] = z;
}
template <typename T> BB_HD void mtv3(T* r, const T* M, const T* v) {  // r = M' v
  T x = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
  T y = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
  T z = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
  r[0] = x; r[1] = y; r[2] = z;
}
template <typename T> BB_HD void mm3(T* r, const T* A, const T* B) {  // r = A B
  T t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = t[i];
}
// packed symmetric 3x3 (xx,yy,zz,xy,xz,yz)
template <typename T> BB_HD void symv(T* r, const T* S, const T* v) {
  T x = S[0] * v[0] + S[3] * v[1] + S[4] * v[2];
  T y = S[3] * v[0] + S[1] * v[1] + S[5] * v[2];
  T z = S[4] * v[0] + S[5] * v[1] + S[2] * v[2];
  r[0] = x; r[1] = y; r[2] = z;
}
template <typename T> BB_HD void sym_rot(T* out, const T* R, const T* S) {  // R S R'
  T F[9] = {S[0], S[3], S[4], S[3], S[1], S[5], S[4], S[5], S[2]};
  T A[9], B[9];
  mm3(A, R, F);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) B[3 * i + j] = A[3 * i] * R[3 * j] + A[3 * i + 1] * R[3 * j + 1] + A[3 * i + 2] * R[3 * j + 2];
  out[0] = B[0]; out[1] = B[4]; out[2] = B[8]; out[3] = B[1]; out[4] = B[2]; out[5] = B[5];
}
template <typename T> BB_HD T clampT(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <typename T> BB_HD T maxT(T a, T b) { return a > b ? a : b; }
// 1/sqrt(x): the device's reciprocal square root; the host test builds divide
template <typename T> BB_HD T rsqrtT(T x) {
#ifdef __HIP_DEVICE_COMPILE__
  return rsqrt(x);
#else
  return T(1) / sqrt(x);
#endif
}
template <typename T> BB_HD T minT(T a, T b) { return a < b ? a : b; }
// Line-search arithmetic (the trial points only steer the search; the solver's
// stopping test and the returned qacc do not depend on these roundings):
// 1/sqrt(x) and a / b from the hardware estimates plus one Newton step
// (relative error ~1e-13 in double) instead of the correctly rounded sequences.
template <typename T> BB_HD T rsqrt_ls(T x) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (sizeof(T) == 8) {
    const double r = __builtin_amdgcn_rsq(x);
    return r * fma(-0.5 * x * r, r, 1.5);
  } else {
    return __builtin_amdgcn_rsqf(x);
  }
#else
  return T(1) / sqrt(x);
#endif
}
template <typename T> BB_HD T div_ls(T a, T b) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (sizeof(T) == 8) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(r, fma(-b, r, 1.0), r);
    return a * r;
  } else {
    return a * __builtin_amdgcn_rcpf(b);
  }
#else
  return a / b;
#endif
}

// quaternion (w,x,y,z)
template <typename T> BB_HD void qmul(T* r, const T* a, const T* b) {
  T w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  T x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  T y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  T z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = w; r[1] = x; r[2] = y; r[3] = z;
}
template <typename T> BB_HD void qnormalize(T* q) {
  T n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < T(1e-15)) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  T inv = T(1) / n;
  q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
}
template <typename T> BB_HD void q2mat(T* m, const T* q) {
  T q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  T q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  T q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33; m[4] = q00 - q11 + q22 - q33; m[8] = q00 - q11 - q22 + q33;
  m[1] = 2 * (q12 - q03); m[2] = 2 * (q13 + q02); m[3] = 2 * (q12 + q03);
  m[5] = 2 * (q23 - q01); m[6] = 2 * (q13 - q02); m[7] = 2 * (q23 + q01);
}
// mju_quatIntegrate: q <- normalize(q) * exp(w*h/2)
template <typename T> BB_HD void quat_integrate(T* q, const T* w, T h) {
  T n = sqrt(dot3(w, w));
  T qr[4] = {1, 0, 0, 0};
  if (n >= T(1e-15)) {
    T ang = h * n, s = sin(ang * T(0.5)) / n;
    qr[0] = cos(ang * T(0.5)); qr[1] = w[0] * s; qr[2] = w[1] * s; qr[3] = w[2] * s;
  }
  qnormalize(q);
  qmul(q, q, qr);
}
// mj_integratePos for this model
template <typename T> BB_HD void integrate_pos(T* q, const T* v, T h) {
  q[0] += h * v[0]; q[1] += h * v[1]; q[2] += h * v[2];
  quat_integrate(q + 3, v + 3, h);
  q[7] += h * v[6]; q[8] += h * v[7]; q[9] += h * v[8];
  q[10] += h * v[9]; q[11] += h * v[10]; q[12] += h * v[11];
  quat_integrate(q + 13, v + 12, h);
}

// packed lower-triangular index
constexpr BB_HD int hidx(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// --------------------------------------------------------- kinematics
template <typename T>
struct Kin {
  T Rb[9], RB[9];      // base / ball orientation (world <- local)
  T pb[3], pB[3];      // base / ball frame origins (world)
  T c[3];              // ball geom centre (world)
  T wc[3][3];          // wheel COM = capsule centre (base-local)
  T Rw[3][9];          // wheel orientation (base-local)
};

template <typename T>
BB_HD void kinematics_base(const ModelT<T>& m, const T* q, Kin<T>& k) {
  T qb[4] = {q[3], q[4], q[5], q[6]};
  qnormalize(qb);
  q2mat(k.Rb, qb);
  T qB[4] = {q[13], q[14], q[15], q[16]};
  qnormalize(qB);
  q2mat(k.RB, qB);
  k.pb[0] = q[0]; k.pb[1] = q[1]; k.pb[2] = q[2];
  k.pB[0] = q[10]; k.pB[1] = q[11]; k.pB[2] = q[12];
  k.c[0] = k.pB[0] + k.RB[2] * m.dz;
  k.c[1] = k.pB[1] + k.RB[5] * m.dz;
  k.c[2] = k.pB[2] + k.RB[8] * m.dz;
}

// wheel w's local frame and COM (the device forward runs one wheel per lane)
template <typename T>
BB_HD void kinematics_wheel(const ModelT<T>& m, const T* q, int w, Kin<T>& k) {
  // xquat_wheel = xquat_base * body_quat * axisangle(axis, theta - theta0)
  T th = q[7 + w] - m.qpos0[7 + w];
  T s = sin(th * T(0.5)), cth = cos(th * T(0.5));
  T ql[4] = {cth, m.axis[0] * s, m.axis[1] * s, m.axis[2] * s};
  T qw[4];
  qmul(qw, m.wq[w], ql);
  qnormalize(qw);
  q2mat(k.Rw[w], qw);
  // origin = anchor - Rw jpos ; COM = origin + Rw cw
  T d[3] = {m.cw[0] - m.jpos[0], m.cw[1] - m.jpos[1], m.cw[2] - m.jpos[2]};
  T t[3];
  mv3(t, k.Rw[w], d);
  k.wc[w][0] = m.anchor[0] + t[0];
  k.wc[w][1] = m.anchor[1] + t[1];
  k.wc[w][2] = m.anchor[2] + t[2];
}

template <typename T>
BB_HD void kinematics(const ModelT<T>& m, const T* q, Kin<T>& k) {
  kinematics_base(m, q, k);
#pragma unroll
  for (int w = 0; w < 3; w++) kinematics_wheel(m, q, w, k);
}

// ------------------------------------------------------------ mass matrix
// Generalised coordinates (MuJoCo free-joint convention): base/ball linear
// velocity in WORLD frame, angular velocity in LOCAL frame, hinge rates.
template <typename T>
struct Mass {
  T mt;            // tree-1 total mass
  T mr[3];         // tree-1 first moment about base origin (base-local)
  T Mtr[9];        // base trans (world) x base rot (local)
  T Mrr[6];        // base rot block (packed sym)
  T Mth[3][3];     // [k] base trans column of hinge k
  T Mrh[3][3];     // [k] base rot column of hinge k
  T Mhh[3];
  T mB;
  T MBtr[9];       // ball trans x ball rot
  T MBrr[3];       // ball rot diagonal (constant)
};

// wheel w's share of the tree-1 mass matrix: its rotated inertia Iw, the hinge
// columns Mth/Mrh/Mhh[w] and its terms of the tree-1 first moment (mrw) and
// inertia about the base origin (IOw); build_mass adds the terms in wheel order
template <typename T>
BB_HD void mass_wheel(const ModelT<T>& m, const Kin<T>& k, int w, Mass<T>& M, T* Iw, T* mrw, T* IOw) {
  const T* c = k.wc[w];
  sym_rot(Iw, k.Rw[w], m.Iw);
  mrw[0] = m.mw * c[0]; mrw[1] = m.mw * c[1]; mrw[2] = m.mw * c[2];
  T cc = dot3(c, c);
  IOw[0] = Iw[0] + m.mw * (cc - c[0] * c[0]);
  IOw[1] = Iw[1] + m.mw * (cc - c[1] * c[1]);
  IOw[2] = Iw[2] + m.mw * (cc - c[2] * c[2]);
  IOw[3] = Iw[3] - m.mw * c[0] * c[1];
  IOw[4] = Iw[4] - m.mw * c[0] * c[2];
  IOw[5] = Iw[5] - m.mw * c[1] * c[2];
  // hinge motion subspace S = (u; anchor x u) about the base origin
  const T* u = m.u[w];
  T ca[3] = {c[0] - m.anchor[0], c[1] - m.anchor[1], c[2] - m.anchor[2]};
  T vc[3];
  cross3(vc, u, ca);                       // wheel COM velocity per unit rate
  T p[3] = {m.mw * vc[0], m.mw * vc[1], m.mw * vc[2]};
  T L[3], t[3];
  symv(L, Iw, u);
  T uIu = dot3(u, L);
  cross3(t, c, p);
  L[0] += t[0]; L[1] += t[1]; L[2] += t[2];  // angular momentum about base origin
  mv3(M.Mth[w], k.Rb, p);
  M.Mrh[w][0] = L[0]; M.Mrh[w][1] = L[1]; M.Mrh[w][2] = L[2];
  M.Mhh[w] = uIu + m.mw * dot3(vc, vc) + m.armature;
}

// the rest of the mass matrix from the wheel terms (mrw[w][3], IOw[w][6])
template <typename T>
BB_HD void mass_finish(const ModelT<T>& m, const Kin<T>& k, Mass<T>& M, const T (*mrw)[3], const T (*IOw)[6]) {
  T mr[3] = {m.h0[0], m.h0[1], m.h0[2]};
  T IO[6] = {m.I0O[0], m.I0O[1], m.I0O[2], m.I0O[3], m.I0O[4], m.I0O[5]};
#pragma unroll
  for (int w = 0; w < 3; w++) {
#pragma unroll
    for (int i = 0; i < 3; i++) mr[i] += mrw[w][i];
#pragma unroll
    for (int i = 0; i < 6; i++) IO[i] += IOw[w][i];
  }
  M.mt = m.m0 + 3 * m.mw;
  M.mr[0] = mr[0]; M.mr[1] = mr[1]; M.mr[2] = mr[2];
  T S[9] = {0, mr[2], -mr[1], -mr[2], 0, mr[0], mr[1], -mr[0], 0};  // -[mr]x
  mm3(M.Mtr, k.Rb, S);
#pragma unroll
  for (int i = 0; i < 6; i++) M.Mrr[i] = IO[i];
  const T dz = m.dz;
  M.mB = m.mB;
  T SB[9] = {0, m.mB * dz, 0, -m.mB * dz, 0, 0, 0, 0, 0};  // -mB [d]x, d = (0,0,dz)
  mm3(M.MBtr, k.RB, SB);
  M.MBrr[0] = m.IB + m.mB * dz * dz;
  M.MBrr[1] = m.IB + m.mB * dz * dz;
  M.MBrr[2] = m.IB;
}

template <typename T>
BB_HD void build_mass(const ModelT<T>& m, const Kin<T>& k, Mass<T>& M, T (&Iw)[3][6]) {
  T mrw[3][3], IOw[3][6];
#pragma unroll
  for (int w = 0; w < 3; w++) mass_wheel(m, k, w, M, Iw[w], mrw[w], IOw[w]);
  mass_finish(m, k, M, mrw, IOw);
}

template <typename T>
BB_HD void mass_mul(const Mass<T>& M, const T* x, T* y) {  // y = M x
  T t[3], r[3];
  mv3(t, M.Mtr, x + 3);
  y[0] = M.mt * x[0] + t[0];
  y[1] = M.mt * x[1] + t[1];
  y[2] = M.mt * x[2] + t[2];
  mtv3(t, M.Mtr, x);
  symv(r, M.Mrr, x + 3);
  y[3] = t[0] + r[0]; y[4] = t[1] + r[1]; y[5] = t[2] + r[2];
#pragma unroll
  for (int w = 0; w < 3; w++) {
    T xh = x[6 + w];
#pragma unroll
    for (int i = 0; i < 3; i++) { y[i] += M.Mth[w][i] * xh; y[3 + i] += M.Mrh[w][i] * xh; }
    y[6 + w] = dot3(M.Mth[w], x) + dot3(M.Mrh[w], x + 3) + M.Mhh[w] * xh;
  }
  mv3(t, M.MBtr, x + 12);
  y[9] = M.mB * x[9] + t[0];
  y[10] = M.mB * x[10] + t[1];
  y[11] = M.mB * x[11] + t[2];
  mtv3(t, M.MBtr, x + 9);
  y[12] = t[0] + M.MBrr[0] * x[12];
  y[13] = t[1] + M.MBrr[1] * x[13];
  y[14] = t[2] + M.MBrr[2] * x[14];
}

template <typename T>
BB_HD void mass_dense(const Mass<T>& M, T* H) {  // packed lower 15x15
#pragma unroll
  for (int i = 0; i < NH; i++) H[i] = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    H[hidx(i, i)] = M.mt;
#pragma unroll
    for (int j = 0; j < 3; j++) H[hidx(3 + i, j)] = M.Mtr[3 * j + i];
  }
  H[hidx(3, 3)] = M.Mrr[0]; H[hidx(4, 4)] = M.Mrr[1]; H[hidx(5, 5)] = M.Mrr[2];
  H[hidx(4, 3)] = M.Mrr[3]; H[hidx(5, 3)] = M.Mrr[4]; H[hidx(5, 4)] = M.Mrr[5];
#pragma unroll
  for (int w = 0; w < 3; w++) {
#pragma unroll
    for (int j = 0; j < 3; j++) { H[hidx(6 + w, j)] = M.Mth[w][j]; H[hidx(6 + w, 3 + j)] = M.Mrh[w][j]; }
    H[hidx(6 + w, 6 + w)] = M.Mhh[w];
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    H[hidx(9 + i, 9 + i)] = M.mB;
#pragma unroll
    for (int j = 0; j < 3; j++) H[hidx(12 + i, 9 + j)] = M.MBtr[3 * j + i];
    H[hidx(12 + i, 12 + i)] = M.MBrr[i];
  }
}

// ------------------------------------------------------------- bias (RNE)
// apply spatial inertia (mass m, COM c, inertia about COM Ic) at the frame
// origin to motion (w; v): p = m (v + w x c), L = Ic w + c x p
template <typename T>
BB_HD void inertia_apply(T m, const T* c, const T* Ic, const T* w, const T* v, T* L, T* p) {
  T t[3];
  cross3(t, w, c);
  p[0] = m * (v[0] + t[0]); p[1] = m * (v[1] + t[1]); p[2] = m * (v[2] + t[2]);
  symv(L, Ic, w);
  cross3(t, c, p);
  L[0] += t[0]; L[1] += t[1]; L[2] += t[2];
}
// f = I A + V xf (I V) for one body (all local coordinates about one origin)
template <typename T>
BB_HD void body_force(T m, const T* c, const T* Ic, const T* Aw, const T* Av, const T* Vw, const T* Vv,
                      T* fa, T* fl) {
  T La[3], pa[3], Lv[3], pv[3], t[3];
  inertia_apply(m, c, Ic, Aw, Av, La, pa);
  inertia_apply(m, c, Ic, Vw, Vv, Lv, pv);
  // V xf (L; p) = (w x L + v x p; w x p)
  cross3(t, Vw, Lv); fa[0] = La[0] + t[0]; fa[1] = La[1] + t[1]; fa[2] = La[2] + t[2];
  cross3(t, Vv, pv); fa[0] += t[0]; fa[1] += t[1]; fa[2] += t[2];
  cross3(t, Vw, pv); fl[0] = pa[0] + t[0]; fl[1] = pa[1] + t[1]; fl[2] = pa[2] + t[2];
}

// tree-1 motion at the base origin (base-local): angular w0, linear vl and the
// spatial acceleration a0 = Rb' (0,0,g) + vl x w0
template <typename T>
BB_HD void bias_base_motion(const ModelT<T>& m, const Kin<T>& k, const T* v, T* w0, T* vl, T* a0) {
  w0[0] = v[3]; w0[1] = v[4]; w0[2] = v[5];
  mtv3(vl, k.Rb, v);
  T t[3];
  cross3(t, vl, w0);
  a0[0] = m.grav * k.Rb[6] + t[0];
  a0[1] = m.grav * k.Rb[7] + t[1];
  a0[2] = m.grav * k.Rb[8] + t[2];
}

// wheel w's RNE force (fa; fl) about the base origin; returns qfrc_bias[6+w]
template <typename T>
BB_HD T bias_wheel(const ModelT<T>& m, const Kin<T>& k, const T* Iw, const T* v, int w, const T* w0, const T* vl,
                   const T* a0, T* fa, T* fl) {
  const T* u = m.u[w];
  T au[3];
  cross3(au, m.anchor, u);           // S = (u; anchor x u)
  T qd = v[6 + w];
  T Vw[3] = {w0[0] + qd * u[0], w0[1] + qd * u[1], w0[2] + qd * u[2]};
  T Vv[3] = {vl[0] + qd * au[0], vl[1] + qd * au[1], vl[2] + qd * au[2]};
  // A = A0 + qd (V0 xm S) ; V0 xm S = (w x u; w x au + v x u)
  T x1[3], x2[3], x3[3];
  cross3(x1, w0, u);
  cross3(x2, w0, au);
  cross3(x3, vl, u);
  T Aw[3] = {qd * x1[0], qd * x1[1], qd * x1[2]};
  T Av[3] = {a0[0] + qd * (x2[0] + x3[0]), a0[1] + qd * (x2[1] + x3[1]), a0[2] + qd * (x2[2] + x3[2])};
  body_force(m.mw, k.wc[w], Iw, Aw, Av, Vw, Vv, fa, fl);
  return dot3(u, fa) + dot3(au, fl);
}

// qfrc_bias from the wheel forces fw[w] = (fa; fl): base composite, the
// wheel sums in wheel order, and the ball (bias[6..8] are set by the caller)
template <typename T>
BB_HD void bias_finish(const ModelT<T>& m, const Kin<T>& k, const T* v, const T (*fw)[6], T* bias) {
  T w0[3], vl[3], a0[3], t[3];
  bias_base_motion(m, k, v, w0, vl, a0);
  const T zero[3] = {0, 0, 0};
  // base composite: mass m0, COM h0/m0, inertia about COM derived from I0O
  T Fa[3], Fl[3];
  {
    T c0[3] = {m.h0[0] / m.m0, m.h0[1] / m.m0, m.h0[2] / m.m0};
    T cc = dot3(c0, c0);
    T Ic[6] = {m.I0O[0] - m.m0 * (cc - c0[0] * c0[0]), m.I0O[1] - m.m0 * (cc - c0[1] * c0[1]),
               m.I0O[2] - m.m0 * (cc - c0[2] * c0[2]), m.I0O[3] + m.m0 * c0[0] * c0[1],
               m.I0O[4] + m.m0 * c0[0] * c0[2], m.I0O[5] + m.m0 * c0[1] * c0[2]};
    body_force(m.m0, c0, Ic, zero, a0, w0, vl, Fa, Fl);
  }
#pragma unroll
  for (int w = 0; w < 3; w++) {
    Fa[0] += fw[w][0]; Fa[1] += fw[w][1]; Fa[2] += fw[w][2];
    Fl[0] += fw[w][3]; Fl[1] += fw[w][4]; Fl[2] += fw[w][5];
  }
  mv3(bias, k.Rb, Fl);
  bias[3] = Fa[0]; bias[4] = Fa[1]; bias[5] = Fa[2];
  // ---- ball, ball-local coordinates about the ball frame origin
  T wB[3] = {v[12], v[13], v[14]};
  T vB[3];
  mtv3(vB, k.RB, v + 9);
  cross3(t, vB, wB);
  T aB[3] = {m.grav * k.RB[6] + t[0], m.grav * k.RB[7] + t[1], m.grav * k.RB[8] + t[2]};
  T cB[3] = {0, 0, m.dz};
  T IcB[6] = {m.IB, m.IB, m.IB, 0, 0, 0};
  T fa[3], fl[3];
  body_force(m.mB, cB, IcB, zero, aB, wB, vB, fa, fl);
  mv3(bias + 9, k.RB, fl);
  bias[12] = fa[0]; bias[13] = fa[1]; bias[14] = fa[2];
}

// qfrc_bias = C(q,v) v + gravity  (mj_rne with flg_acc = 0)
template <typename T>
BB_HD void bias_forces(const ModelT<T>& m, const Kin<T>& k, const T (&Iw)[3][6], const T* v, T* bias) {
  T w0[3], vl[3], a0[3], fw[3][6];
  bias_base_motion(m, k, v, w0, vl, a0);
#pragma unroll
  for (int w = 0; w < 3; w++) bias[6 + w] = bias_wheel(m, k, Iw[w], v, w, w0, vl, a0, fw[w], fw[w] + 3);
  bias_finish(m, k, v, fw, bias);
}

// ------------------------------------------------------------- contacts
// getImpedance with solimp (dmin, dmax, width, mid, power), clamped to
// [mjMINIMP, mjMAXIMP] (engine_core_constraint.c)
template <typename T>
BB_HD T impedance(const ModelT<T>& m, T pos) {
  T x = pos / m.solimp[2];
  if (x < 0) x = -x;
  if (x >= T(1) || x <= T(0)) return x >= T(1) ? m.solimp[1] : m.solimp[0];
  T y;
  const T mid = m.solimp[3];
  if (x <= mid) y = x * x / mid;                     // power 2: x^p / mid^(p-1)
  else y = T(1) - (T(1) - x) * (T(1) - x) / (T(1) - mid);
  return m.solimp[0] + y * (m.solimp[1] - m.solimp[0]);
}

// mju_makeFrame for a frame whose second axis is undefined (hfield contacts)
template <typename T>
BB_HD void frame_from_normal(const T* n, T* t1, T* t2) {
  T y[3] = {0, 0, 0};
  if (fabs(n[1]) < T(0.5)) y[1] = 1; else y[2] = 1;
  T d = dot3(n, y);
  t1[0] = y[0] - d * n[0]; t1[1] = y[1] - d * n[1]; t1[2] = y[2] - d * n[2];
  T inv = rsqrtT(dot3(t1, t1));
  t1[0] *= inv; t1[1] *= inv; t1[2] *= inv;
  cross3(t2, n, t1);
}

// elliptic condim-3 cone: cost zones of mj_constraintUpdate.  Returns force
// (= -d cost / d jar) and optionally the 3x3 Hessian (packed sym xx,yy,zz,xy,xz,yz).
template <typename T>
BB_HD void cone_eval(const T* jar, T mu, T f1, T f2, const T* D, T* force, T* C) {
  T U0 = jar[0] * mu, U1 = jar[1] * f1, U2 = jar[2] * f2;
  T N = U0, Tn = sqrt(U1 * U1 + U2 * U2);
  if (N >= mu * Tn || (Tn <= 0 && N >= 0)) {          // top zone: separated
    force[0] = force[1] = force[2] = 0;
    if (C) { C[0] = C[1] = C[2] = C[3] = C[4] = C[5] = 0; }
  } else if (mu * N + Tn <= 0 || (Tn <= 0 && N < 0)) {  // bottom zone: quadratic
    force[0] = -D[0] * jar[0]; force[1] = -D[1] * jar[1]; force[2] = -D[2] * jar[2];
    if (C) { C[0] = D[0]; C[1] = D[1]; C[2] = D[2]; C[3] = C[4] = C[5] = 0; }
  } else {                                               // middle zone: cone
    T Dm = D[0] / (mu * mu * (1 + mu * mu));
    T g = N - mu * Tn;
    T iT = T(1) / Tn;
    T gr[3] = {mu, -mu * f1 * U1 * iT, -mu * f2 * U2 * iT};
    T s = -Dm * g;
    force[0] = s * gr[0]; force[1] = s * gr[1]; force[2] = s * gr[2];
    if (C) {
      T k = Dm * g * (-mu) * iT;   // Dm g d2g, d2g = -mu f f' (I/T - U U'/T^3)
      T iT2 = iT * iT;
      C[0] = Dm * gr[0] * gr[0];
      C[1] = Dm * gr[1] * gr[1] + k * f1 * f1 * (T(1) - U1 * U1 * iT2);
      C[2] = Dm * gr[2] * gr[2] + k * f2 * f2 * (T(1) - U2 * U2 * iT2);
      C[3] = Dm * gr[0] * gr[1];
      C[4] = Dm * gr[0] * gr[2];
      C[5] = Dm * gr[1] * gr[2] - k * f1 * f2 * U1 * U2 * iT2;
    }
  }
}

// One ball-wheel contact (explicit pair, condim 3).  Jacobian rows over the
// 13 structural columns: base trans (3), base rot (3), hinge w, ball trans (3),
// ball rot (3) -- see wheel_col().
template <typename T>
struct WheelCon {
  T J[3][13];     // rows: normal, axle tangent (patch), drive tangent
  T aref[3], D[3];
};

// global dof index of wheel-contact column i for wheel w
BB_HD constexpr int wheel_col(int i, int w) { return i < 6 ? i : (i == 6 ? 6 + w : i + 2); }

// ground-contact store: element (slot s, field f) at base[(s*NGF + f)*stride]
template <typename T>
struct GStore {
  T* base;
  int stride;
  BB_HD T& at(int s, int f) const { return base[(s * NGF + f) * stride]; }
};

// patched mjraw_SphereCapsule (tools/mujoco_fix.patch:11-16) + mju_makeFrame
template <typename T>
BB_HD void wheel_contact(const ModelT<T>& m, const Kin<T>& k, const T* v, int w, WheelCon<T>& C) {
  T t[3], gp[3], ax[3], axl[3];
  mv3(t, k.Rb, k.wc[w]);
  gp[0] = k.pb[0] + t[0]; gp[1] = k.pb[1] + t[1]; gp[2] = k.pb[2] + t[2];
  mv3(axl, k.Rw[w], m.gz);
  mv3(ax, k.Rb, axl);
  T vec[3] = {k.c[0] - gp[0], k.c[1] - gp[1], k.c[2] - gp[2]};
  T x = clampT(dot3(ax, vec), -m.wheel_hh, m.wheel_hh);
  T dif[3] = {gp[0] + ax[0] * x - k.c[0], gp[1] + ax[1] * x - k.c[1], gp[2] + ax[2] * x - k.c[2]};
  T cd = sqrt(dot3(dif, dif));
  T dist = cd - m.ball_r - m.wheel_r;
  const T act = dist <= 0 ? T(1) : T(0);
  T n[3];
  if (cd > 0) { T ic = T(1) / cd; n[0] = dif[0] * ic; n[1] = dif[1] * ic; n[2] = dif[2] * ic; }
  else { n[0] = 1; n[1] = 0; n[2] = 0; }
  // frame row 2 = capsule axis (patch), orthogonalised; row 3 = n x t1
  T dn = dot3(n, ax);
  T t1[3] = {ax[0] - dn * n[0], ax[1] - dn * n[1], ax[2] - dn * n[2]};
  T it1 = T(1) / sqrt(dot3(t1, t1));
  t1[0] *= it1; t1[1] *= it1; t1[2] *= it1;
  T t2[3];
  cross3(t2, n, t1);
  T pos[3];
  T sp = m.ball_r + dist * T(0.5);
  pos[0] = k.c[0] + n[0] * sp; pos[1] = k.c[1] + n[1] * sp; pos[2] = k.c[2] + n[2] * sp;
  T lb[3] = {pos[0] - k.pb[0], pos[1] - k.pb[1], pos[2] - k.pb[2]};
  mv3(t, k.Rb, m.anchor);
  T la[3] = {lb[0] - t[0], lb[1] - t[1], lb[2] - t[2]};
  T lB[3] = {pos[0] - k.pB[0], pos[1] - k.pB[1], pos[2] - k.pB[2]};
  T uw[3];
  mv3(uw, k.Rb, m.u[w]);
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const T* d = r == 0 ? n : (r == 1 ? t1 : t2);
    T x1[3], br[3];
    C.J[r][0] = d[0]; C.J[r][1] = d[1]; C.J[r][2] = d[2];
    cross3(x1, lb, d);
    mtv3(br, k.Rb, x1);
    C.J[r][3] = br[0]; C.J[r][4] = br[1]; C.J[r][5] = br[2];
    cross3(x1, la, d);
    C.J[r][6] = dot3(uw, x1);
    C.J[r][7] = -d[0]; C.J[r][8] = -d[1]; C.J[r][9] = -d[2];
    cross3(x1, lB, d);
    mtv3(t, k.RB, x1);
    C.J[r][10] = -t[0]; C.J[r][11] = -t[1]; C.J[r][12] = -t[2];
  }
  // impedance, R, D (elliptic, impratio = 1) and aref
  T imp = clampT(impedance(m, dist), T(0.0001), T(0.9999));
  T tran = m.iw_ball + m.iw_wheel[w];
  T R0 = maxT(T(1e-15), (1 - imp) * tran / imp);
  T rr = m.fr_wheel[0] / m.fr_wheel[1];
  T R2 = R0 * rr * rr;
  C.D[0] = act / R0; C.D[1] = act / R0; C.D[2] = act / R2;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    T vel = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) vel += C.J[r][i] * v[wheel_col(i, w)];
    C.aref[r] = (C.D[0] > 0 ? T(1) : T(0)) * (-m.Bd * vel - (r == 0 ? m.K * imp * dist : T(0)));
  }
}

// J x for one wheel contact row
template <typename T>
BB_HD T wheel_row_mul(const WheelCon<T>& C, int w, int r, const T* x) {
  T acc = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) acc += C.J[r][i] * x[wheel_col(i, w)];
  return acc;
}

// closest point on triangle (Ericson, RTCD 5.1.5) -- used for the top face
template <typename T>
BB_HD void closest_pt_tri(T* res, const T* p, const T* a, const T* b, const T* c) {
  T ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  T ac[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  T ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  T d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { res[0] = a[0]; res[1] = a[1]; res[2] = a[2]; return; }
  T bp[3] = {p[0] - b[0], p[1] - b[1], p[2] - b[2]};
  T d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { res[0] = b[0]; res[1] = b[1]; res[2] = b[2]; return; }
  T vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    T vv = d1 / (d1 - d3);
    res[0] = a[0] + vv * ab[0]; res[1] = a[1] + vv * ab[1]; res[2] = a[2] + vv * ab[2];
    return;
  }
  T cp[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
  T d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { res[0] = c[0]; res[1] = c[1]; res[2] = c[2]; return; }
  T vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    T ww = d2 / (d2 - d6);
    res[0] = a[0] + ww * ac[0]; res[1] = a[1] + ww * ac[1]; res[2] = a[2] + ww * ac[2];
    return;
  }
  T va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    T ww = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    res[0] = b[0] + ww * (c[0] - b[0]); res[1] = b[1] + ww * (c[1] - b[1]); res[2] = b[2] + ww * (c[2] - b[2]);
    return;
  }
  T den = T(1) / (va + vb + vc), vv = vb * den, ww = vc * den;
  res[0] = a[0] + ab[0] * vv + ac[0] * ww;
  res[1] = a[1] + ab[1] * vv + ac[1] * ww;
  res[2] = a[2] + ab[2] * vv + ac[2] * ww;
}

// Exact sphere vs triangular prism (top vertices V, bottom plane zb): the
// minimum-translation penetration that mjc_ConvexHField's convex solver
// converges to.  Fast path when the sphere centre is above the whole top face
// (closest feature is on the top triangle); general path otherwise.
template <typename T>
BB_HD bool sphere_prism(const T* c, T r, const T V[3][3], T zb, T* n, T* dist) {
  T zmax = maxT(V[0][2], maxT(V[1][2], V[2][2]));
  T q[3];
  if (c[2] >= zmax) {
    closest_pt_tri(q, c, V[0], V[1], V[2]);
  } else {
    // inside test
    T area = (V[1][0] - V[0][0]) * (V[2][1] - V[0][1]) - (V[2][0] - V[0][0]) * (V[1][1] - V[0][1]);
    T sg = area > 0 ? T(1) : T(-1);
    bool inside = c[2] >= zb;
    T edist[3], eo[3][2];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const T* P = V[i];
      const T* Q = V[(i + 1) % 3];
      T ex = Q[0] - P[0], ey = Q[1] - P[1];
      T cr = ex * (c[1] - P[1]) - ey * (c[0] - P[0]);
      if (cr * sg < 0) inside = false;
      T nx = ey * sg, ny = -ex * sg, nl = sqrt(nx * nx + ny * ny);
      eo[i][0] = nx / nl; eo[i][1] = ny / nl;
      edist[i] = fabs(cr) / nl;
    }
    T e1[3] = {V[1][0] - V[0][0], V[1][1] - V[0][1], V[1][2] - V[0][2]};
    T e2[3] = {V[2][0] - V[0][0], V[2][1] - V[0][1], V[2][2] - V[0][2]};
    T nt[3];
    cross3(nt, e1, e2);
    if (nt[2] < 0) { nt[0] = -nt[0]; nt[1] = -nt[1]; nt[2] = -nt[2]; }
    T inl = T(1) / sqrt(dot3(nt, nt));
    nt[0] *= inl; nt[1] *= inl; nt[2] *= inl;
    T dtop = dot3(nt, V[0]) - dot3(nt, c);
    if (inside && dtop >= 0) {
      T best = dtop;
      n[0] = nt[0]; n[1] = nt[1]; n[2] = nt[2];
      if (c[2] - zb < best) { best = c[2] - zb; n[0] = 0; n[1] = 0; n[2] = -1; }
#pragma unroll
      for (int i = 0; i < 3; i++)
        if (edist[i] < best) { best = edist[i]; n[0] = eo[i][0]; n[1] = eo[i][1]; n[2] = 0; }
      *dist = -best - r;
      return true;
    }
    // outside: closest point over the 5 faces (8 triangles)
    T B[3][3] = {{V[0][0], V[0][1], zb}, {V[1][0], V[1][1], zb}, {V[2][0], V[2][1], zb}};
    T best = T(1e30);
#pragma unroll
    for (int f = 0; f < 8; f++) {
      const T* a;
      const T* b;
      const T* cc;
      switch (f) {
        case 0: a = V[0]; b = V[1]; cc = V[2]; break;
        case 1: a = B[0]; b = B[1]; cc = B[2]; break;
        case 2: a = V[0]; b = V[1]; cc = B[1]; break;
        case 3: a = V[0]; b = B[1]; cc = B[0]; break;
        case 4: a = V[1]; b = V[2]; cc = B[2]; break;
        case 5: a = V[1]; b = B[2]; cc = B[1]; break;
        case 6: a = V[2]; b = V[0]; cc = B[0]; break;
        default: a = V[2]; b = B[0]; cc = B[2]; break;
      }
      T qq[3];
      closest_pt_tri(qq, c, a, b, cc);
      T dd[3] = {c[0] - qq[0], c[1] - qq[1], c[2] - qq[2]};
      T d2 = dot3(dd, dd);
      if (d2 < best) { best = d2; q[0] = qq[0]; q[1] = qq[1]; q[2] = qq[2]; }
    }
  }
  T dd[3] = {c[0] - q[0], c[1] - q[1], c[2] - q[2]};
  T d = sqrt(dot3(dd, dd));
  if (d > r) return false;
  if (d > T(1e-12)) { T id = T(1) / d; n[0] = dd[0] * id; n[1] = dd[1] * id; n[2] = dd[2] * id; }
  else {
    T e1[3] = {V[1][0] - V[0][0], V[1][1] - V[0][1], V[1][2] - V[0][2]};
    T e2[3] = {V[2][0] - V[0][0], V[2][1] - V[0][1], V[2][2] - V[0][2]};
    cross3(n, e1, e2);
    if (n[2] < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    T inl = T(1) / sqrt(dot3(n, n));
    n[0] *= inl; n[1] *= inl; n[2] *= inl;
  }
  *dist = d - r;
  return true;
}

// Stored ground contact -> Jacobian rows (normal, t1, t2) over the ball dofs
// (world-linear F_r, local-angular RB'(lever x F_r)), aref and D.  RB: ball
// orientation, v: the stage velocity (qvel) the constraint is built at.
template <typename T>
BB_HD void ground_contact(const ModelT<T>& m, const T* gc, const T* RB, const T* v, T (&J)[3][6], T (&aref)[3],
                          T& D) {
  const T n[3] = {gc[GF_N], gc[GF_N + 1], gc[GF_N + 2]};
  const T dist = gc[GF_DIST];
  // lever = (ball geom centre - ball frame origin) - n (r + dist/2)
  const T sp = m.ball_r + dist * T(0.5);
  const T lv[3] = {m.dz * RB[2] - n[0] * sp, m.dz * RB[5] - n[1] * sp, m.dz * RB[8] - n[2] * sp};
  T t1[3], t2[3];
  frame_from_normal(n, t1, t2);
  const T* F[3] = {n, t1, t2};
#pragma unroll
  for (int r = 0; r < 3; r++) {
    T x1[3], x2[3];
    cross3(x1, lv, F[r]);
    mtv3(x2, RB, x1);
#pragma unroll
    for (int i = 0; i < 3; i++) { J[r][i] = F[r][i]; J[r][3 + i] = x2[i]; }
  }
  const T imp = clampT(impedance(m, dist), T(0.0001), T(0.9999));
  D = minT(T(1e15), imp / ((1 - imp) * m.iw_ball));  // 1 / max(1e-15, (1 - imp) iw / imp), one divide
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const T vel = J[r][0] * v[9] + J[r][1] * v[10] + J[r][2] * v[11] + J[r][3] * v[12] + J[r][4] * v[13] +
                  J[r][5] * v[14];
    aref[r] = -m.Bd * vel - (r == 0 ? m.K * imp * dist : T(0));
  }
}

// Persistent body poses the solve needs after the kinematics scratch is reused.
template <typename T>
struct Poses {
  T Rb[9], pb[3], RB[9], pB[3];
};

// Stored base-tree contact in world form.  Its 13-column Jacobian (the
// wheel-contact layout: base lin 3, base ang 3, hinge 1, ball lin 3, ball ang 3)
// is J[r][q] = F_r . w_q with F = (n, t1, t2) and one world vector per column:
//   base lin i   e_i                      base ang i   Rb_i x db
//   hinge        hw = uw x da             ball lin i   -ball e_i
//   ball ang i   -ball RB_i x dB
// (Rb_i, RB_i: body axes, db/dB: contact point from the base/ball origins, uw
// and da: the wheel's hinge axis and the point from the hinge anchor), so
// J x = F V(x) with V(x) = x_lin + (Rb x_ang) x db + hw x_h - ball (x_blin +
// (RB x_bang) x dB) (body_V), and J' C J = W' (F' C F) W: the solve broadcasts
// A = F' C F and phi = F' f instead of J.  aref and D: isotropic friction,
// mu = 1 (mj_makeImpedance / mj_instantiateContact).
template <typename T>
struct BodyFrame {
  T F[3][3], db[3], dB[3], hw[3], aref[3], D, ball;
  int hinge;  // wheel of the hinge column (-1: none)
};

// V(x) of a body contact (see BodyFrame): J x = F V(x)
template <typename T>
BB_HD void body_V(const BodyFrame<T>& b, const Poses<T>& P, const T* x, T (&V)[3]) {
  T om[3], wx[3];
  mv3(om, P.Rb, x + 3);
  cross3(wx, om, b.db);
  const T xh = b.hinge >= 0 ? hinge_sel(b.hinge, x) : T(0);
  T ob[3], bx[3];
  mv3(ob, P.RB, x + 12);
  cross3(bx, ob, b.dB);
#pragma unroll
  for (int i = 0; i < 3; i++) V[i] = x[i] + wx[i] + b.hw[i] * xh - b.ball * (x[9 + i] + bx[i]);
}

// stored contact (BF_* fields) -> BodyFrame at the stage velocity v
template <typename T>
BB_HD void body_frame(const ModelT<T>& m, const T* bc, const Poses<T>& P, const T* v, BodyFrame<T>& b) {
  const int code = int(bc[BF_CODE]);
  const int b1 = code >> 3, b2 = code & 7;
  const T n[3] = {bc[BF_N], bc[BF_N + 1], bc[BF_N + 2]};
  const T dist = bc[BF_DIST];
  T t1[3], t2[3];
  frame_from_normal(n, t1, t2);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    b.F[0][i] = n[i]; b.F[1][i] = t1[i]; b.F[2][i] = t2[i];
    b.db[i] = bc[BF_P + i] - P.pb[i];
    b.dB[i] = bc[BF_P + i] - P.pB[i];
    b.hw[i] = 0;
  }
  b.hinge = (b2 >= 4 && b2 <= 6) ? b2 - 4 : -1;
  if (b.hinge >= 0) {
    T uw[3], t[3], da[3];
    mv3(uw, P.Rb, m.u[b.hinge]);
    mv3(t, P.Rb, m.anchor);
    da[0] = b.db[0] - t[0]; da[1] = b.db[1] - t[1]; da[2] = b.db[2] - t[2];
    cross3(b.hw, uw, da);
  }
  b.ball = b1 == 7 ? T(1) : T(0);
  const T iw2 = b2 == 1 ? m.iw_base : (b2 <= 3 ? m.iw_cam[b2 - 2] : m.iw_wheel[b2 - 4]);
  const T tran = iw2 + (b1 == 7 ? m.iw_ball : T(0));
  const T imp = clampT(impedance(m, dist), T(0.0001), T(0.9999));
  b.D = T(1) / maxT(T(1e-15), (1 - imp) * tran / imp);
  T V[3];
  body_V(b, P, v, V);
#pragma unroll
  for (int r = 0; r < 3; r++) b.aref[r] = -m.Bd * dot3(b.F[r], V) - (r == 0 ? m.K * imp * dist : T(0));
}

// line-search terms of a body contact: per row r, jar0_r = J_r a - aref_r and
// J_r s; D returned
template <typename T>
BB_HD void body_ls_terms(const ModelT<T>& m, const T* bc, const Poses<T>& P, const T* v, const T* a, const T* s,
                         T (&c6)[6], T& D) {
  BodyFrame<T> b;
  body_frame(m, bc, P, v, b);
  T Va[3], Vs[3];
  body_V(b, P, a, Va);
  body_V(b, P, s, Vs);
#pragma unroll
  for (int r = 0; r < 3; r++) {
    c6[r] = dot3(b.F[r], Va) - b.aref[r];
    c6[3 + r] = dot3(b.F[r], Vs);
  }
  D = b.D;
}

// mjc_ConvexHField for the ball: sub-grid from the ball AABB, triangular
// prisms in MuJoCo's sliding-window order, one contact per penetrated prism.
// Writes normal/lever/aref/D into the store; returns the contact count.
template <typename T>
BB_HD int collide_ground(const ModelT<T>& m, const Kin<T>& k, const T* v, const float* hf, T size_z,
                         const GStore<T>& st, int* overflow) {
  const T r = m.ball_r;
  const T* c = k.c;
  const T sx = m.hf_sx, sy = m.hf_sy, zb = m.hf_bottom;
  T xmin = c[0] - r, xmax = c[0] + r, ymin = c[1] - r, ymax = c[1] + r, zmin = c[2] - r, zmax = c[2] + r;
  if (!(xmin <= sx && xmax >= -sx && ymin <= sy && ymax >= -sy && zmin <= size_z && zmax >= -zb)) return 0;
  const int N1 = HF_N - 1;
  int cmin = (int)floor((xmin + sx) / (2 * sx) * N1);
  int cmax = (int)ceil((xmax + sx) / (2 * sx) * N1);
  int rmin = (int)floor((ymin + sy) / (2 * sy) * N1);
  int rmax = (int)ceil((ymax + sy) / (2 * sy) * N1);
  cmin = cmin < 0 ? 0 : cmin;
  cmax = cmax > N1 ? N1 : cmax;
  rmin = rmin < 0 ? 0 : rmin;
  rmax = rmax > N1 ? N1 : rmax;
  const T dx = 2 * sx / N1, dy = 2 * sy / N1;
  (void)v;
  int ng = 0;
  for (int rr = rmin; rr < rmax; rr++) {
    T W[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    int nvert = 0;
    const T y0 = dy * rr - sy, y1 = dy * (rr + 1) - sy;
    for (int cc = cmin; cc <= cmax; cc++) {
      const T x = dx * cc - sx;
      const T z0 = T(hf[rr * HF_N + cc]) * size_z;
      const T z1 = T(hf[(rr + 1) * HF_N + cc]) * size_z;
#pragma unroll
      for (int i = 0; i < 2; i++) {
#pragma unroll
        for (int j = 0; j < 3; j++) { W[0][j] = W[1][j]; W[1][j] = W[2][j]; }
        W[2][0] = x; W[2][1] = i ? y1 : y0; W[2][2] = i ? z1 : z0;
        nvert++;
        if (nvert <= 2) continue;
        if (W[0][2] < zmin && W[1][2] < zmin && W[2][2] < zmin) continue;
        // conservative reject: distance to the prism's xy box and top height
        T bx0 = minT(W[0][0], minT(W[1][0], W[2][0])), bx1 = maxT(W[0][0], maxT(W[1][0], W[2][0]));
        T by0 = minT(W[0][1], minT(W[1][1], W[2][1])), by1 = maxT(W[0][1], maxT(W[1][1], W[2][1]));
        T ztop = maxT(W[0][2], maxT(W[1][2], W[2][2]));
        T ex = maxT(T(0), maxT(bx0 - c[0], c[0] - bx1));
        T ey = maxT(T(0), maxT(by0 - c[1], c[1] - by1));
        T ez = maxT(T(0), c[2] - ztop);
        if (ex * ex + ey * ey + ez * ez > r * r) continue;
        T nn[3], dist;
        if (!sphere_prism(c, r, W, -zb, nn, &dist)) continue;
        if (ng >= MAXG) { *overflow = 1; continue; }
#pragma unroll
        for (int i = 0; i < 3; i++) st.at(ng, GF_N + i) = nn[i];
        st.at(ng, GF_DIST) = dist;
        ng++;
      }
    }
  }
  return ng;
}

// ------------------------------------------------------------ Newton solve
template <typename T> BB_HD T eps_of();
template <> BB_HD float eps_of<float>() { return 1.1920929e-7f; }
template <> BB_HD double eps_of<double>() { return 2.220446049250313e-16; }
template <typename T> BB_HD T pivot_eps();
template <> BB_HD float pivot_eps<float>() { return 1e-6f; }
template <> BB_HD double pivot_eps<double>() { return 1e-14; }

// In-place packed Cholesky.  A pivot that roundoff drives below eps*H_jj
// (fp32 with the 1e6x stiffer drive-direction rows) is floored relative to
// the diagonal, so the Newton direction stays finite; descent is then
// enforced by the line search.
template <typename T>
BB_HD void chol_packed(T* H) {
  for (int j = 0; j < NV; j++) {
    const int rj = j * (j + 1) / 2;
    T s = H[rj + j];
    const T floor_j = pivot_eps<T>() * maxT(s, T(1e-30));
    for (int k = 0; k < j; k++) s -= H[rj + k] * H[rj + k];
    s = s > floor_j ? s : floor_j;
    const T d = sqrt(s), id = T(1) / d;
    H[rj + j] = d;
    for (int i = j + 1; i < NV; i++) {
      const int ri = i * (i + 1) / 2;
      T t = H[ri + j];
      for (int k = 0; k < j; k++) t -= H[ri + k] * H[rj + k];
      H[ri + j] = t * id;
    }
  }
}
template <typename T>
BB_HD void chol_solve_packed(const T* L, T* x) {
  // x lives in registers: unrolled over i, rolled over nothing dynamic
#pragma unroll
  for (int i = 0; i < NV; i++) {
    T s = x[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[hidx(i, k)] * x[k];
    x[i] = s / L[hidx(i, i)];
  }
#pragma unroll
  for (int i = NV - 1; i >= 0; i--) {
    T s = x[i];
#pragma unroll
    for (int k = i + 1; k < NV; k++) s -= L[hidx(k, i)] * x[k];
    x[i] = s / L[hidx(i, i)];
  }
}

}  // namespace bb
