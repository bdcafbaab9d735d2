// Test-only host build of the product's per-env templates (bb_step.h), used
// to debug the kernel math against the oracle on a machine without a GPU.
// Never shipped, never loaded by the product path.
#include <math.h>
#include <random>
#include <vector>
#include "bb_bodycon.h"
#include "bb_model.h"
#include "bb_step.h"
#include "bb_pairmap.h"

using namespace bb;

#include <stdlib.h>
template <typename T>
static ModelT<T> model_for(int fp64) {
  SolverCfg sc = default_solver(fp64 != 0);
  if (getenv("BB_TOL")) sc.tol = atof(getenv("BB_TOL"));
  if (getenv("BB_STEPREL")) sc.step_rel = atof(getenv("BB_STEPREL"));
  if (getenv("BB_LSTOL")) sc.ls_tol = atof(getenv("BB_LSTOL"));
  if (getenv("BB_MAXIT")) sc.maxiter = atoi(getenv("BB_MAXIT"));
  ModelT<double> d = compile_model(sc);
  return cast_model<T>(d);
}

template <typename T>
static int fwd(const double* q, const double* v, const double* ctrl, double* acc, const float* hf, double size_z,
               int fp64, double* extra) {
  ModelT<T> m = model_for<T>(fp64);
  T qq[NQ], vv[NV], cc[3], aa[NV];
  for (int i = 0; i < NQ; i++) qq[i] = T(q[i]);
  for (int i = 0; i < NV; i++) { vv[i] = T(v[i]); aa[i] = T(acc[i]); }
  for (int i = 0; i < 3; i++) cc[i] = T(ctrl[i]);
  static EnvWork<T> W;
  StageOut<T> so;
  int it = forward(m, qq, vv, cc, aa, TerrainRef<T>{hf, T(size_z), T(1e30)}, W, &so, Team{1, 0});
  for (int i = 0; i < NV; i++) acc[i] = double(aa[i]);
  if (extra) {
    extra[0] = so.ng; extra[1] = so.iters; extra[2] = so.overflow;
    for (int i = 0; i < 3; i++) { extra[3 + i] = so.w_world[i]; extra[6 + i] = so.v_com[i]; }
  }
  return it;
}

template <typename T>
static int envstep(const EnvCfg* cfg, double* q, double* v, double* w, int* step, const float* a, const float* hf,
                   double size_z, float* obs, float* rew, float* pos2d, int fp64) {
  ModelT<T> m = model_for<T>(fp64);
  T qq[NQ], vv[NV], ww[NV];
  for (int i = 0; i < NQ; i++) qq[i] = T(q[i]);
  for (int i = 0; i < NV; i++) { vv[i] = T(v[i]); ww[i] = T(w[i]); }
  static EnvWork<T> W;
  int it = 0;
  int fl = env_step(m, *cfg, qq, vv, ww, *step, a, TerrainRef<T>{hf, T(size_z), T(1e30)}, W, obs, *rew, pos2d, &it, Team{1, 0});
  for (int i = 0; i < NQ; i++) q[i] = double(qq[i]);
  for (int i = 0; i < NV; i++) { v[i] = double(vv[i]); w[i] = double(ww[i]); }
  return fl | (it << 8);
}

// random unit vector / rotation helpers for the geometry checks
static void rand_unit(std::mt19937_64& g, double* a) {
  std::normal_distribution<double> N(0, 1);
  double l = 0;
  for (int i = 0; i < 3; i++) { a[i] = N(g); l += a[i] * a[i]; }
  l = sqrt(l);
  for (int i = 0; i < 3; i++) a[i] /= l;
}
static void rand_rot(std::mt19937_64& g, double* R) {
  std::normal_distribution<double> N(0, 1);
  double q[4], l = 0;
  for (int i = 0; i < 4; i++) { q[i] = N(g); l += q[i] * q[i]; }
  l = sqrt(l);
  for (int i = 0; i < 4; i++) q[i] /= l;
  q2mat(R, q);
}

extern "C" {
// BodyFrame / body_V (bb_physics.h) against the base-tree contact Jacobian
// written column by column (base lin e_i, base ang Rb'(db x F_r), hinge
// uw.(da x F_r), ball -F_r, ball ang -RB'(dB x F_r)): max |J x - F V(x)| over
// n random contacts, poses and x.
double hc_body_jacobian_check(int n, unsigned seed) {
  ModelT<double> m = compile_model(default_solver(true));
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> U(-1, 1);
  double worst = 0;
  for (int it = 0; it < n; it++) {
    Poses<double> P;
    rand_rot(g, P.Rb);
    rand_rot(g, P.RB);
    for (int i = 0; i < 3; i++) { P.pb[i] = U(g) * 0.3; P.pB[i] = U(g) * 0.3; }
    double bc[NBF], nrm[3];
    rand_unit(g, nrm);
    for (int i = 0; i < 3; i++) { bc[BF_N + i] = nrm[i]; bc[BF_P + i] = U(g) * 0.4; }
    bc[BF_DIST] = -0.005 * (U(g) + 1);
    const int b1 = (it % 3 == 0) ? 7 : 0, b2 = 1 + it % 6;  // ball or hfield x tower/sticks/wheels
    bc[BF_CODE] = double(8 * b1 + b2);
    double v[NV], x[NV];
    for (int i = 0; i < NV; i++) { v[i] = U(g); x[i] = U(g); }
    BodyFrame<double> b;
    body_frame(m, bc, P, v, b);
    double V[3];
    body_V(b, P, x, V);
    // explicit columns
    const double db[3] = {bc[BF_P] - P.pb[0], bc[BF_P + 1] - P.pb[1], bc[BF_P + 2] - P.pb[2]};
    const double dB[3] = {bc[BF_P] - P.pB[0], bc[BF_P + 1] - P.pB[1], bc[BF_P + 2] - P.pB[2]};
    const int hinge = (b2 >= 4 && b2 <= 6) ? b2 - 4 : -1;
    double uw[3] = {0, 0, 0}, da[3] = {0, 0, 0};
    if (hinge >= 0) {
      double t[3];
      mv3(uw, P.Rb, m.u[hinge]);
      mv3(t, P.Rb, m.anchor);
      for (int i = 0; i < 3; i++) da[i] = db[i] - t[i];
    }
    const double ball = b1 == 7 ? 1.0 : 0.0;
    for (int r = 0; r < 3; r++) {
      const double* F = b.F[r];
      double J[13], x1[3], x2[3];
      for (int i = 0; i < 3; i++) J[i] = F[i];
      cross3(x1, db, F);
      mtv3(x2, P.Rb, x1);
      for (int i = 0; i < 3; i++) J[3 + i] = x2[i];
      cross3(x1, da, F);
      J[6] = hinge >= 0 ? dot3(uw, x1) : 0.0;
      for (int i = 0; i < 3; i++) J[7 + i] = -ball * F[i];
      cross3(x1, dB, F);
      mtv3(x2, P.RB, x1);
      for (int i = 0; i < 3; i++) J[10 + i] = -ball * x2[i];
      double jx = 0;
      for (int q = 0; q < 6; q++) jx += J[q] * x[q];
      jx += hinge >= 0 ? J[6] * x[6 + hinge] : 0.0;
      for (int q = 7; q < 13; q++) jx += J[q] * x[q + 2];
      worst = fmax(worst, fabs(jx - dot3(F, V)));
    }
  }
  return worst;
}

// capsule_prism_apart (bb_bodycon.h) against the minimum over the prism's 8
// boundary triangles (seg_tri, the oracle's form) for n random segments that
// miss one hfield cell's prism: returns the count of differing contact
// decisions, *worst the largest difference in distance, normal or position.
int hc_capsule_apart_check(int n, unsigned seed, double* worst) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> U(-1, 1);
  int mism = 0;
  *worst = 0;
  const int tri[8][3] = {{0, 1, 2}, {3, 4, 5}, {0, 1, 4}, {0, 4, 3}, {1, 2, 5}, {1, 5, 4}, {2, 0, 3}, {2, 3, 5}};
  for (int it = 0; it < n; it++) {
    const double s = 0.03425, x0 = U(g) * 0.1, y0 = U(g) * 0.1;
    double px[3] = {x0, x0, x0 + s}, py[3] = {y0, y0 + s, y0}, Tp[3][3];
    if (it & 1) { px[0] = x0; py[0] = y0 + s; px[1] = x0 + s; py[1] = y0; px[2] = x0 + s; py[2] = y0 + s; }
    const bool flat = it & 2;
    for (int i = 0; i < 3; i++) { Tp[i][0] = px[i]; Tp[i][1] = py[i]; Tp[i][2] = flat ? 0.0 : 0.05 + 0.02 * U(g); }
    PrismG<double> P;
    prism_build(P, Tp, -0.1);
    Seg<double> sg;
    for (int i = 0; i < 3; i++) sg.c[i] = i < 2 ? x0 + s / 2 + U(g) * 0.06 : (flat ? 0.02 + 0.01 * U(g) : 0.06 + U(g) * 0.06);
    rand_unit(g, sg.a);
    sg.hh = 0.02 + 0.05 * (U(g) + 1);
    sg.r = 0.025;
    double p0[3], p1[3];
    seg_ends(sg, p0, p1);
    const double dir[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    double t0 = 0, t1 = 1;
    bool inter = true;
    for (int f = 0; f < 5; f++) {
      const double a0 = dot3(P.pn[f], p0) - P.pd[f], ad = dot3(P.pn[f], dir);
      if (fabs(ad) < 1e-30) { if (a0 > 0) inter = false; }
      else { const double t = -a0 / ad; if (ad > 0) t1 = fmin(t1, t); else t0 = fmax(t0, t); }
    }
    if (t0 > t1) inter = false;
    if (inter) continue;
    double d1 = 0, n1[3], q1[3];
    const bool h1 = capsule_prism_apart(sg, P, p0, p1, d1, n1, q1);
    double best = 1e30, bp[3] = {0, 0, 0}, bq[3] = {0, 0, 0};
    for (int f = 0; f < 8; f++) {
      double cp[3], cq[3];
      const double d = seg_tri(p0, p1, P.V[tri[f][0]], P.V[tri[f][1]], P.V[tri[f][2]], cp, cq);
      if (d < best) { best = d; for (int i = 0; i < 3; i++) { bp[i] = cp[i]; bq[i] = cq[i]; } }
    }
    const bool h2 = best < sg.r;
    if (h1 != h2) { mism++; continue; }
    if (!h1) continue;
    double n2[3], q2[3];
    if (best > 1e-12) { for (int i = 0; i < 3; i++) n2[i] = (bp[i] - bq[i]) / best; }
    else { n2[0] = P.pn[0][0]; n2[1] = P.pn[0][1]; n2[2] = P.pn[0][2]; }
    const double d2 = best - sg.r;
    for (int i = 0; i < 3; i++) q2[i] = bp[i] - n2[i] * (sg.r + d2 * 0.5);
    double e = fabs(d1 - d2);
    for (int i = 0; i < 3; i++) e = fmax(e, fmax(fabs(n1[i] - n2[i]), fabs(q1[i] - q2[i])));
    *worst = fmax(*worst, e);
  }
  return mism;
}

int hc_forward(const double* q, const double* v, const double* ctrl, double* acc, const float* hf, double size_z,
               int fp64, double* extra) {
  return fp64 ? fwd<double>(q, v, ctrl, acc, hf, size_z, 1, extra) : fwd<float>(q, v, ctrl, acc, hf, size_z, 0, extra);
}
int hc_env_step(const EnvCfg* cfg, double* q, double* v, double* w, int* step, const float* a, const float* hf,
                double size_z, float* obs, float* rew, float* pos2d, int fp64) {
  return fp64 ? envstep<double>(cfg, q, v, w, step, a, hf, size_z, obs, rew, pos2d, 1)
              : envstep<float>(cfg, q, v, w, step, a, hf, size_z, obs, rew, pos2d, 0);
}
void hc_model(double* out) {
  ModelT<double> m = compile_model(default_solver(true));
  out[0] = m.m0; out[1] = m.mw; out[2] = m.mB; out[3] = m.iw_ball;
  out[4] = m.iw_wheel[0]; out[5] = m.iw_wheel[1]; out[6] = m.iw_wheel[2]; out[7] = 1.0 / (m.scale * 15);
  out[8] = m.iw_base; out[9] = m.iw_cam[0]; out[10] = m.iw_cam[1];
  for (int i = 0; i < 3; i++) { out[11 + i] = m.stick_c[0][i]; out[14 + i] = m.stick_a[0][i]; out[17 + i] = m.stick_c[1][i]; out[20 + i] = m.stick_a[1][i]; }
}
// the relief pair's block -> (kind, index within kind) map (bb_pairmap.h)
int hc_pair_kind_of(int b, int nf, int ns, int* wg) { return pair_kind_of(b, nf, ns, wg); }
}
