// bb_model.h -- host-side compiler of ballbot.xml into bb::ModelT.
//
// Replaces mujoco.MjModel.from_xml_path (ballbot_env.py:261) for the one model
// this framework simulates: geometry, inertia-from-geoms (mjCBody inertia,
// capsule/cylinder/box/sphere formulas), hinge frames, contact-pair
// parameters, and mj_setConst's body_invweight0 / stat.meaninertia (computed
// here with this framework's own mass matrix, bb_physics.h).
#pragma once

#include <math.h>
#include <string.h>

#include "bb_physics.h"

namespace bb {

namespace detail {
inline void euler_quat(double* q, double ax, double ay, double az) {  // MJCF "xyz" intrinsic, degrees
  const double pi = 3.14159265358979323846;
  double e[3] = {ax * pi / 180, ay * pi / 180, az * pi / 180};
  q[0] = 1; q[1] = q[2] = q[3] = 0;
  for (int i = 0; i < 3; i++) {
    double r[4] = {cos(e[i] / 2), 0, 0, 0};
    r[1 + i] = sin(e[i] / 2);
    qmul(q, q, r);
  }
}
// accumulate a geom (mass m at pos, inertia diag I in frame R) into mass, first moment, inertia about origin
inline void accum(double m, const double* pos, const double* R, const double* I, double& ms, double* h, double* IO) {
  double S[6] = {I[0], I[1], I[2], 0, 0, 0}, Sr[6];
  sym_rot(Sr, R, S);
  double p2 = dot3(pos, pos);
  IO[0] += Sr[0] + m * (p2 - pos[0] * pos[0]);
  IO[1] += Sr[1] + m * (p2 - pos[1] * pos[1]);
  IO[2] += Sr[2] + m * (p2 - pos[2] * pos[2]);
  IO[3] += Sr[3] - m * pos[0] * pos[1];
  IO[4] += Sr[4] - m * pos[0] * pos[2];
  IO[5] += Sr[5] - m * pos[1] * pos[2];
  ms += m;
  h[0] += m * pos[0]; h[1] += m * pos[1]; h[2] += m * pos[2];
}
inline void capsule(double rho, double r, double hh, double& m, double* I) {
  const double pi = 3.14159265358979323846, h = 2 * hh;
  double ms = rho * 4.0 / 3.0 * pi * r * r * r, mc = rho * pi * r * r * h;
  m = ms + mc;
  I[0] = I[1] = mc * (3 * r * r + h * h) / 12 + ms * (0.4 * r * r + 0.25 * h * h + 0.375 * h * r);
  I[2] = mc * r * r / 2 + ms * 0.4 * r * r;
}
}  // namespace detail

struct SolverCfg {
  double tol, ls_tol, step_rel;
  int maxiter, ls_maxiter;
};

inline SolverCfg default_solver(bool fp64) {
  // MuJoCo: tolerance 1e-8, iterations 100, ls_iterations 50.  The minimiser is
  // unique, so the fp32 build stops at its roundoff floor instead.
  if (fp64) return SolverCfg{1e-8, 1e-2, 1e-14, 100, 50};  // MuJoCo tolerance / ls_tolerance / iterations
  return SolverCfg{2e-6, 1e-3, 3e-7, 16, 16};
}

// mjModel.opt overrides (bb_params.opt_timestep / opt_disableflags): the step
// size and MuJoCo's mjDSBL_PASSIVE / mjDSBL_GRAVITY switches, for the physics
// invariants of SURVEY.md §8 C1 (RK4 order, momentum conservation).  Defaults:
// ballbot.xml's 0.002 s, everything enabled.
struct OptCfg {
  double timestep = 0.002;
  int disable = 0;  // BB_DSBL_PASSIVE (32), BB_DSBL_GRAVITY (64): MuJoCo's bit values
};

// Compile ballbot.xml (values cited per line) into a double-precision model.
inline ModelT<double> compile_model(const SolverCfg& sc, const OptCfg& opt = OptCfg{}) {
  using namespace detail;
  const double pi = 3.14159265358979323846;
  ModelT<double> m;
  memset(&m, 0, sizeof m);
  const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  // ---- base body (ballbot.xml:38-42): tower cylinder + ballast box
  double ms = 0, h[3] = {0, 0, 0}, IO[6] = {0, 0, 0, 0, 0, 0};
  {
    double r = 0.11, hh = 0.14, rho = 23.6;
    double mc = rho * pi * r * r * 2 * hh;
    double Ic[3] = {mc * (3 * r * r + 4 * hh * hh) / 12, mc * (3 * r * r + 4 * hh * hh) / 12, mc * r * r / 2};
    double p[3] = {0, 0, 0.2};
    accum(mc, p, I3, Ic, ms, h, IO);
    double a = 0.1, mb = 400.0 * 8 * a * a * a, Ib = mb * (2 * a * a) / 3;
    double Ibx[3] = {Ib, Ib, Ib}, pb[3] = {0, 0, 0.002};
    accum(mb, pb, I3, Ibx, ms, h, IO);
  }
  // ---- camera bodies (ballbot.xml:44-54), welded: capsule sticks (fromto
  // (0,0,0)->(-+0.2,0,0), r 0.01, density 1000).  The cone meshes reference
  // meshes/cone.stl, absent from the reference (.gitignore:178): massless.
  for (int cam = 0; cam < 2; cam++) {
    double bq[4], R[9];
    euler_quat(bq, 180, cam == 0 ? -30 : 30, 0);
    q2mat(R, bq);
    double bp[3] = {cam == 0 ? 0.17 : -0.17, -0.01, -0.06};
    double mcap, Icap[3];
    capsule(1000.0, 0.01, 0.1, mcap, Icap);
    // stick axis along body x: inertia about its centre in body frame
    double lp[3] = {cam == 0 ? -0.1 : 0.1, 0, 0}, p[3];
    mv3(p, R, lp);
    p[0] += bp[0]; p[1] += bp[1]; p[2] += bp[2];
    // geom frame: z along x-axis of the body -> R_body * Rz2x
    double Rg[9] = {0, 0, 1, 0, 1, 0, -1, 0, 0};  // columns: x->-z, y->y, z->x
    double RR[9];
    mm3(RR, R, Rg);
    accum(mcap, p, RR, Icap, ms, h, IO);
  }
  m.m0 = ms;
  for (int i = 0; i < 3; i++) m.h0[i] = h[i];
  // collision geometry of the base tree (base frame)
  m.tower_c[0] = 0; m.tower_c[1] = 0; m.tower_c[2] = 0.2; m.tower_r = 0.11; m.tower_hh = 0.14;
  m.stick_r = 0.01; m.stick_hh = 0.1;
  double cam_com[2][3];
  for (int cam = 0; cam < 2; cam++) {
    double bq[4], R[9], lp[3] = {cam == 0 ? -0.1 : 0.1, 0, 0}, p[3], ex[3] = {1, 0, 0};
    euler_quat(bq, 180, cam == 0 ? -30 : 30, 0);
    q2mat(R, bq);
    mv3(p, R, lp);
    m.stick_c[cam][0] = p[0] + (cam == 0 ? 0.17 : -0.17);
    m.stick_c[cam][1] = p[1] - 0.01;
    m.stick_c[cam][2] = p[2] - 0.06;
    mv3(m.stick_a[cam], R, ex);
    for (int i = 0; i < 3; i++) cam_com[cam][i] = m.stick_c[cam][i];
  }
  // base body's own COM (tower + ballast; the sticks are the cam bodies' mass)
  double base_com[3];
  {
    const double r = 0.11, hh = 0.14, mc = 23.6 * pi * r * r * 2 * hh, mb = 400.0 * 8 * 0.001;
    for (int i = 0; i < 3; i++) base_com[i] = 0;
    base_com[2] = (mc * 0.2 + mb * 0.002) / (mc + mb);
  }
  for (int i = 0; i < 6; i++) m.I0O[i] = IO[i];
  // ---- wheels (ballbot.xml:56-70): capsule r .025 hh .02 density 620,
  // euler (-45, 9, 0) at (-0.018,-0.08,-0.053); hinge at (0,0,0.0293)
  {
    double gq[4], Rg[9], Ic[3];
    euler_quat(gq, -45, 9, 0);
    q2mat(Rg, gq);
    capsule(620.0, 0.025, 0.02, m.mw, Ic);
    double S[6] = {Ic[0], Ic[1], Ic[2], 0, 0, 0};
    sym_rot(m.Iw, Rg, S);
    m.cw[0] = -0.018; m.cw[1] = -0.08; m.cw[2] = -0.053;
    m.gz[0] = Rg[2]; m.gz[1] = Rg[5]; m.gz[2] = Rg[8];
    double ax[3] = {-0.15316554764123935, -0.6903189805903613, -0.7071067953657663};
    double n = sqrt(dot3(ax, ax));
    for (int i = 0; i < 3; i++) m.axis[i] = ax[i] / n;
    m.jpos[0] = 0; m.jpos[1] = 0; m.jpos[2] = 0.0293;
    m.anchor[0] = 0; m.anchor[1] = 0; m.anchor[2] = -0.001 + 0.0293;
    for (int k = 0; k < 3; k++) {
      euler_quat(m.wq[k], 0, 0, 120.0 * k);
      double R[9];
      q2mat(R, m.wq[k]);
      mv3(m.u[k], R, m.axis);
    }
    m.wheel_r = 0.025; m.wheel_hh = 0.02;
    m.armature = 0.005; m.damping = (opt.disable & 32) ? 0.0 : 0.8;  // mjDSBL_PASSIVE drops the joint damping
  }
  // ---- ball (ballbot.xml:76-79): sphere r .09 density 55 at (0,0,-0.14)
  m.ball_r = 0.09;
  m.mB = 55.0 * 4.0 / 3.0 * pi * 0.09 * 0.09 * 0.09;
  m.IB = 0.4 * m.mB * 0.09 * 0.09;
  m.dz = -0.14;
  // ---- options (ballbot.xml:3-5) + MuJoCo defaults
  m.h = opt.timestep;
  m.grav = (opt.disable & 64) ? 0.0 : 9.81;  // mjDSBL_GRAVITY
  m.hf_sx = 5; m.hf_sy = 5; m.hf_bottom = 0.1;  // hfield size (ballbot.xml:23)
  m.solimp[0] = 0.9; m.solimp[1] = 0.95; m.solimp[2] = 0.001; m.solimp[3] = 0.5; m.solimp[4] = 2;
  {
    double dmax = 0.95, tc = fmax(0.02, 2 * m.h), dr = 1.0;  // solref (0.02, 1), refsafe
    m.K = 1 / fmax(1e-15, dmax * dmax * tc * tc * dr * dr);
    m.Bd = 2 / fmax(1e-15, dmax * tc);
  }
  m.fr_wheel[0] = 0.001; m.fr_wheel[1] = 1.0;
  for (int i = 0; i < NQ; i++) m.qpos0[i] = 0;
  m.qpos0[2] = 0.24; m.qpos0[3] = 1;   // base pos (ballbot.xml:38)
  m.qpos0[12] = 0.26; m.qpos0[13] = 1; // ball pos (ballbot.xml:76)
  m.tol = sc.tol; m.ls_tol = sc.ls_tol; m.step_rel2 = sc.step_rel * sc.step_rel;
  m.maxiter = sc.maxiter; m.ls_maxiter = sc.ls_maxiter;

  // ---- mj_setConst at qpos0: meaninertia, body_invweight0
  Kin<double> k;
  kinematics(m, m.qpos0, k);
  Mass<double> M;
  double Iw_[3][6];
  build_mass(m, k, M, Iw_);
  static double H[NH];
  mass_dense(M, H);
  double tr = 0;
  for (int i = 0; i < NV; i++) tr += H[hidx(i, i)];
  m.scale = 1.0 / (tr / NV * NV);
  chol_packed(H);
  // translational invweight at a point rigid with the base (base frame offset)
  auto invweight_base = [&](const double* lp) {
    double Jp[3][NV];
    memset(Jp, 0, sizeof Jp);
    double l[3];
    mv3(l, k.Rb, lp);
    for (int i = 0; i < 3; i++) Jp[i][i] = 1;
    for (int j = 0; j < 3; j++) {
      double e[3] = {k.Rb[j], k.Rb[3 + j], k.Rb[6 + j]}, x[3];
      cross3(x, e, l);
      for (int i = 0; i < 3; i++) Jp[i][3 + j] = x[i];
    }
    double s = 0;
    for (int i = 0; i < 3; i++) {
      double x[NV];
      for (int d = 0; d < NV; d++) x[d] = Jp[i][d];
      chol_solve_packed(H, x);
      for (int d = 0; d < NV; d++) s += Jp[i][d] * x[d];
    }
    return s / 3;
  };
  // translational invweight at a body COM: trace(Jp M^-1 Jp')/3
  auto invweight = [&](int body) {
    double Jp[3][NV];
    memset(Jp, 0, sizeof Jp);
    double p[3];
    if (body == 7) {
      p[0] = k.c[0]; p[1] = k.c[1]; p[2] = k.c[2];
      double l[3] = {p[0] - k.pB[0], p[1] - k.pB[1], p[2] - k.pB[2]};
      for (int i = 0; i < 3; i++) Jp[i][9 + i] = 1;
      for (int j = 0; j < 3; j++) {
        double e[3] = {k.RB[j], k.RB[3 + j], k.RB[6 + j]}, x[3];
        cross3(x, e, l);
        for (int i = 0; i < 3; i++) Jp[i][12 + j] = x[i];
      }
    } else {
      int w = body - 4;
      double t[3];
      mv3(t, k.Rb, k.wc[w]);
      p[0] = k.pb[0] + t[0]; p[1] = k.pb[1] + t[1]; p[2] = k.pb[2] + t[2];
      double l[3] = {p[0] - k.pb[0], p[1] - k.pb[1], p[2] - k.pb[2]};
      for (int i = 0; i < 3; i++) Jp[i][i] = 1;
      for (int j = 0; j < 3; j++) {
        double e[3] = {k.Rb[j], k.Rb[3 + j], k.Rb[6 + j]}, x[3];
        cross3(x, e, l);
        for (int i = 0; i < 3; i++) Jp[i][3 + j] = x[i];
      }
      double uw[3], a[3], la[3], x[3];
      mv3(uw, k.Rb, m.u[w]);
      mv3(a, k.Rb, m.anchor);
      la[0] = l[0] - a[0]; la[1] = l[1] - a[1]; la[2] = l[2] - a[2];
      cross3(x, uw, la);
      for (int i = 0; i < 3; i++) Jp[i][6 + w] = x[i];
    }
    double s = 0;
    for (int i = 0; i < 3; i++) {
      double x[NV];
      for (int d = 0; d < NV; d++) x[d] = Jp[i][d];
      chol_solve_packed(H, x);
      for (int d = 0; d < NV; d++) s += Jp[i][d] * x[d];
    }
    return s / 3;
  };
  m.iw_ball = invweight(7);
  for (int w = 0; w < 3; w++) m.iw_wheel[w] = invweight(4 + w);
  m.iw_base = invweight_base(base_com);
  m.iw_cam[0] = invweight_base(cam_com[0]);
  m.iw_cam[1] = invweight_base(cam_com[1]);
  return m;
}

template <typename T>
inline ModelT<T> cast_model(const ModelT<double>& d) {
  ModelT<T> m;
  const double* src = reinterpret_cast<const double*>(&d);
  // ModelT is all-T except the two ints (maxiter, ls_maxiter): copy field by field
#define BBC(x) m.x = T(d.x)
#define BBA(x, n) for (int i = 0; i < n; i++) m.x[i] = T(d.x[i])
  BBC(m0); BBA(h0, 3); BBA(I0O, 6); BBC(mw); BBA(cw, 3); BBA(Iw, 6); BBA(gz, 3);
  for (int k = 0; k < 3; k++) { BBA(wq[k], 4); BBA(u[k], 3); }
  BBA(axis, 3); BBA(jpos, 3); BBA(anchor, 3);
  BBC(wheel_r); BBC(wheel_hh); BBC(armature); BBC(damping);
  BBC(mB); BBC(IB); BBC(ball_r); BBC(dz);
  BBA(tower_c, 3); BBC(tower_r); BBC(tower_hh); BBA(stick_c[0], 3); BBA(stick_c[1], 3);
  BBA(stick_a[0], 3); BBA(stick_a[1], 3); BBC(stick_r); BBC(stick_hh);
  BBC(iw_base); BBA(iw_cam, 2);
  BBC(iw_ball); BBA(iw_wheel, 3); BBC(K); BBC(Bd); BBA(solimp, 5); BBA(fr_wheel, 2);
  BBC(h); BBC(grav); BBC(hf_sx); BBC(hf_sy); BBC(hf_bottom); BBC(scale); BBC(tol); BBC(ls_tol); BBC(step_rel2);
  m.maxiter = d.maxiter; m.ls_maxiter = d.ls_maxiter;
  BBA(qpos0, NQ);
#undef BBC
#undef BBA
  (void)src;
  return m;
}

}  // namespace bb
