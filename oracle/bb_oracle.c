/*
 * bb_oracle.c -- CPU fp64 restatement of the reference's hot path:
 *   `mujoco.mj_step(model, data)` for ballbot_gym/models/ballbot.xml with the
 *   tools/mujoco_fix.patch contact frame, and the BBotSimulation.step glue.
 *
 * TEST INFRASTRUCTURE ONLY (see bb_oracle.h).  This is the parity checker;
 * the shipped HIP path lives in openballbot-rl_amd/csrc and never calls it.
 *
 * Physics parity vs. real MuJoCo: UNPINNED (MuJoCo is not in /root/reference
 * and cannot be built or imported here).  The algorithms
 * below follow MuJoCo's published pipeline and are deliberately written in
 * MuJoCo's *general* form (tree loops, com-based spatial vectors, dense J,
 * dense Newton) so that they are independent of the specialised GPU kernel:
 *   kinematics        mj_kinematics            (engine_core_smooth.c)
 *   com/cinert/cdof   mj_comPos
 *   mass matrix       sum_b J_b' I_b J_b (== mj_crb result)
 *   cvel/cdof_dot     mj_comVel
 *   bias              mj_rne(flg_acc=0)
 *   passive/actuator  hinge damping (ballbot.xml:58), motor gear 1 (:84-86)
 *   collision         mjraw_SphereCapsule + mujoco_fix.patch:11-16 frame,
 *                     mju_makeFrame, mjc_ConvexHField prism decomposition
 *   constraint        mj_instantiateContact / mj_makeImpedance (elliptic)
 *   solver            Newton on the primal cost (mj_solNewton); the minimiser
 *                     is unique (M > 0), so any convergent method reproduces it
 *   integrator        mj_RungeKutta(N=4) + mj_advance + mj_integratePos
 *   env glue          ballbot_env.py:897-1036 (obs A10, reward A12, term A13)
 */
#include "bb_oracle.h"

/* phase marks for the FLOP-counting build (oracle/flopcount.cpp); no-ops here:
 * 0 kinematics, mass matrix, velocities, bias; 1 collision; 2 constraint
 * assembly (Jacobians, impedance, aref); 3 Newton solver; 4 RK4/glue */
#ifndef BBO_PHASE
#define BBO_PHASE(k) ((void)0)
#endif

#include <math.h>
#include <string.h>
#include <float.h>
#include <stdlib.h>
#include <stdio.h>

#define NQ BBO_NQ
#define NV BBO_NV
#define NB BBO_NBODY
#define MJMINVAL 1e-15
#define MJMINIMP 0.0001
#define MJMAXIMP 0.9999

static const double PI = 3.14159265358979323846;

/* ------------------------------------------------------------------ options */
static int g_flags = 0;
static int g_maxiter = 100;          /* MuJoCo default opt.iterations */
static double g_tol = 1e-8;          /* MuJoCo default opt.tolerance */
/* line search: MuJoCo's PrimalSearch (newton() below) with opt.ls_tolerance and
 * opt.ls_iterations; converged when |phi'| < tolerance * ls_tolerance * |s| / scale */
static double g_lstol = 0.01;        /* MuJoCo default opt.ls_tolerance */
static int g_lsmax = 50;             /* MuJoCo default opt.ls_iterations */

int bbo_abi_version(void) { return 3; }
void bbo_set_flags(int flags) { g_flags = flags; }
int bbo_get_flags(void) { return g_flags; }
void bbo_set_solver(int maxiter, double tol) { g_maxiter = maxiter; g_tol = tol; }
void bbo_set_linesearch(int ls_iterations, double ls_tolerance) { g_lsmax = ls_iterations; g_lstol = ls_tolerance; }
/* opt.timestep (the RK4 convergence test; 0 restores ballbot.xml's 0.002) */
static double TIMESTEP = 0.002;
void bbo_set_timestep(double h) { TIMESTEP = h > 0 ? h : 0.002; }

/* ------------------------------------------------------------- small maths */
static void v3copy(double* r, const double* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
static void v3add(double* r, const double* a, const double* b) { for (int i = 0; i < 3; i++) r[i] = a[i] + b[i]; }
static void v3sub(double* r, const double* a, const double* b) { for (int i = 0; i < 3; i++) r[i] = a[i] - b[i]; }
static void v3scl(double* r, const double* a, double s) { for (int i = 0; i < 3; i++) r[i] = a[i] * s; }
static double v3dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double v3norm(const double* a) { return sqrt(v3dot(a, a)); }
static void v3cross(double* r, const double* a, const double* b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  v3copy(r, t);
}
static double v3normalize(double* a) {
  double n = v3norm(a);
  if (n < MJMINVAL) { a[0] = 1; a[1] = 0; a[2] = 0; return 0; }
  v3scl(a, a, 1.0 / n);
  return n;
}
/* 3x3 row-major */
static void m3v(double* r, const double* m, const double* v) {
  double t[3];
  for (int i = 0; i < 3; i++) t[i] = m[3 * i] * v[0] + m[3 * i + 1] * v[1] + m[3 * i + 2] * v[2];
  v3copy(r, t);
}
static inline void m3tv(double* r, const double* m, const double* v) {
  double t[3];
  for (int i = 0; i < 3; i++) t[i] = m[i] * v[0] + m[3 + i] * v[1] + m[6 + i] * v[2];
  v3copy(r, t);
}
static void m3mul(double* r, const double* a, const double* b) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof t);
}
static void m3mulT(double* r, const double* a, const double* b) { /* a * b' */
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[3 * j] + a[3 * i + 1] * b[3 * j + 1] + a[3 * i + 2] * b[3 * j + 2];
  memcpy(r, t, sizeof t);
}
/* quaternions (w,x,y,z) */
static void qmul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof t);
}
static void qnormalize(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MJMINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static void q2mat(double* m, const double* q) { /* mju_quat2Mat */
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    memset(m, 0, 9 * sizeof(double)); m[0] = m[4] = m[8] = 1; return;
  }
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33; m[4] = q00 - q11 + q22 - q33; m[8] = q00 - q11 - q22 + q33;
  m[1] = 2 * (q12 - q03); m[2] = 2 * (q13 + q02); m[3] = 2 * (q12 + q03);
  m[5] = 2 * (q23 - q01); m[6] = 2 * (q13 - q02); m[7] = 2 * (q23 + q01);
}
static void axisangle2quat(double* q, const double* axis, double angle) {
  if (angle == 0) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  double s = sin(angle * 0.5);
  q[0] = cos(angle * 0.5); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
/* MJCF euler, degrees, default eulerseq "xyz" (intrinsic): q = qx*qy*qz */
static void euler2quat(double* q, double ax, double ay, double az) {
  double e[3] = {ax * PI / 180, ay * PI / 180, az * PI / 180};
  q[0] = 1; q[1] = q[2] = q[3] = 0;
  for (int i = 0; i < 3; i++) {
    double r[4] = {cos(e[i] / 2), 0, 0, 0};
    r[1 + i] = sin(e[i] / 2);
    qmul(q, q, r);
  }
}
/* mju_quatIntegrate: q <- normalize(q) * exp(vel*scale/2) */
static void quat_integrate(double* q, const double* vel, double scale) {
  double axis[3] = {vel[0], vel[1], vel[2]};
  double angle = scale * v3normalize(axis);
  double qrot[4];
  axisangle2quat(qrot, axis, angle);
  qnormalize(q);
  qmul(q, q, qrot);
}

/* ------------------------------------------------------------ model table */
/* ballbot.xml:38-79.  Body 0 world, 1 base, 2 cam_0_body, 3 cam_1_body,
 * 4..6 wheel_0..2, 7 ball. */
static const int body_parent[NB] = {-1, 0, 1, 1, 1, 1, 1, 0};
static const int body_root[NB] = {0, 1, 1, 1, 1, 1, 1, 7};
static const double HINGE_AXIS[3] = {-0.15316554764123935, -0.6903189805903613, -0.7071067953657663};
static const double HINGE_POS[3] = {0, 0, 0.0293};           /* ballbot.xml:58 */
static const double HINGE_ARMATURE = 0.005, HINGE_DAMPING = 0.8;
static const double BALL_R = 0.09, BALL_RHO = 55.0;           /* ballbot.xml:78 */
static const double BALL_GPOS[3] = {0, 0, -0.14};
static const double WHEEL_R = 0.025, WHEEL_HH = 0.02, WHEEL_RHO = 620.0; /* :57 */
static const double WHEEL_GPOS[3] = {-0.018, -0.08, -0.053};
static const double HF_SIZE[4] = {5, 5, 2.0, 0.1};            /* ballbot.xml:23 */
/* TIMESTEP: ballbot.xml:3, 0.002 (defined with the options above; bbo_set_timestep) */
static const double GRAVITY = 9.81;                           /* MuJoCo default */

typedef struct {
  int compiled;
  double body_pos[NB][3], body_quat[NB][4];
  double mass[NB], ipos[NB][3], inertia[NB][9]; /* full tensor about COM, body frame */
  double jnt_axis[3];                            /* normalised hinge axis */
  double wheel_gquat[4], wheel_gmat[9];          /* wheel capsule orientation in wheel frame */
  double qpos0[NQ];
  double invweight_tran[NB], invweight_rot[NB];
  double meaninertia;
  double ball_mass;
} Model;
static Model M_;

static void add_geom_inertia(int b, double m, const double* pos, const double* gmat, const double* Idiag,
                             double* msum, double* mcom, double* Isum_origin) {
  /* accumulate mass, first moment and inertia about the BODY ORIGIN */
  double Ig[9], tmp[9], D[9] = {Idiag[0], 0, 0, 0, Idiag[1], 0, 0, 0, Idiag[2]};
  m3mul(tmp, gmat, D); m3mulT(Ig, tmp, gmat);
  double p2 = v3dot(pos, pos);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Isum_origin[3 * i + j] += Ig[3 * i + j] + m * ((i == j ? p2 : 0) - pos[i] * pos[j]);
  *msum += m;
  for (int i = 0; i < 3; i++) mcom[i] += m * pos[i];
  (void)b;
}

static void capsule_inertia(double rho, double r, double hh, double* m, double* I) {
  double h = 2 * hh;
  double ms = rho * 4.0 / 3.0 * PI * r * r * r, mc = rho * PI * r * r * h;
  *m = ms + mc;
  I[0] = I[1] = mc * (3 * r * r + h * h) / 12 + ms * (0.4 * r * r + 0.25 * h * h + 0.375 * h * r);
  I[2] = mc * r * r / 2 + ms * 0.4 * r * r;
}

static void z2mat(double* R, const double* vec) { /* mjuu_z2quat then quat2mat */
  double z[3] = {0, 0, 1}, axis[3], v[3] = {vec[0], vec[1], vec[2]}, q[4];
  v3normalize(v);
  v3cross(axis, z, v);
  double s = v3normalize(axis);
  if (s < 1e-10) { axis[0] = 1; axis[1] = 0; axis[2] = 0; }
  double ang = atan2(s, v[2]);
  axisangle2quat(q, axis, ang);
  q2mat(R, q);
}

static void finish_body(int b, double msum, const double* mcom, const double* Iorig) {
  Model* m = &M_;
  m->mass[b] = msum;
  if (msum <= 0) { memset(m->ipos[b], 0, 3 * sizeof(double)); memset(m->inertia[b], 0, 9 * sizeof(double)); return; }
  double c[3]; v3scl(c, mcom, 1.0 / msum);
  v3copy(m->ipos[b], c);
  double c2 = v3dot(c, c);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) m->inertia[b][3 * i + j] = Iorig[3 * i + j] - msum * ((i == j ? c2 : 0) - c[i] * c[j]);
}

static void kinematics_all(const double* qpos, double xpos[NB][3], double xquat[NB][4], double xmat[NB][9],
                           double xipos[NB][3], double xI[NB][9], double xanchor[3][3], double xaxis[3][3]);
static void build_M(const double xmat[NB][9], const double xpos[NB][3], const double xipos[NB][3],
                    const double xI[NB][9], const double xanchor[3][3], const double xaxis[3][3],
                    double subtree_com[NB][3], double cinert[NB][36], double cdof[NV][6], double* Mout);
static int chol(double* A, int n);
static void chol_solve(const double* L, int n, double* x);

static void compile_model(void) {
  Model* m = &M_;
  if (m->compiled) return;
  memset(m, 0, sizeof *m);
  double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  /* body frames (ballbot.xml:38,44,50,56,61,67,76) */
  for (int b = 0; b < NB; b++) { m->body_quat[b][0] = 1; }
  m->body_pos[1][2] = 0.24;
  m->body_pos[2][0] = 0.17; m->body_pos[2][1] = -0.01; m->body_pos[2][2] = -0.06;
  euler2quat(m->body_quat[2], 180, -30, 0);
  m->body_pos[3][0] = -0.17; m->body_pos[3][1] = -0.01; m->body_pos[3][2] = -0.06;
  euler2quat(m->body_quat[3], 180, 30, 0);
  for (int k = 0; k < 3; k++) {
    m->body_pos[4 + k][2] = -0.001;
    euler2quat(m->body_quat[4 + k], 0, 0, 120.0 * k);
  }
  m->body_pos[7][2] = 0.26;
  v3copy(m->jnt_axis, HINGE_AXIS);
  v3normalize(m->jnt_axis);
  euler2quat(m->wheel_gquat, -45, 9, 0);
  q2mat(m->wheel_gmat, m->wheel_gquat);

  /* inertia from geoms (mjCBody inertia from geoms; compiler inertiagrouprange 0..5) */
  {
    /* base: tower cylinder (:41) + ballast box (:42, contype 0 but has mass) */
    double ms = 0, mc[3] = {0}, Io[9] = {0};
    double r = 0.11, hh = 0.14, rho = 23.6;
    double mcyl = rho * PI * r * r * 2 * hh;
    double Icyl[3] = {mcyl * (3 * r * r + 4 * hh * hh) / 12, mcyl * (3 * r * r + 4 * hh * hh) / 12, mcyl * r * r / 2};
    double p1[3] = {0, 0, 0.2};
    add_geom_inertia(1, mcyl, p1, I3, Icyl, &ms, mc, Io);
    double a = 0.1, mb = 400.0 * 8 * a * a * a;
    double Ibox[3] = {mb * (a * a + a * a) / 3, mb * (a * a + a * a) / 3, mb * (a * a + a * a) / 3};
    double p2[3] = {0, 0, 0.002};
    add_geom_inertia(1, mb, p2, I3, Ibox, &ms, mc, Io);
    finish_body(1, ms, mc, Io);
  }
  for (int c = 0; c < 2; c++) {
    /* cam_k_stick capsule fromto (0,0,0)->(-+0.2,0,0), r 0.01, density 1000 (:46,:52).
     * cam_k_geom is a mesh whose asset (meshes/cone.stl) is absent from the
     * reference (.gitignore:178): treated as massless, non-colliding. */
    double ms = 0, mc[3] = {0}, Io[9] = {0};
    double to[3] = {c == 0 ? -0.2 : 0.2, 0, 0};
    double pos[3] = {to[0] / 2, 0, 0}, R[9], mcap, Icap[3];
    z2mat(R, to);
    capsule_inertia(1000.0, 0.01, 0.1, &mcap, Icap);
    add_geom_inertia(2 + c, mcap, pos, R, Icap, &ms, mc, Io);
    finish_body(2 + c, ms, mc, Io);
  }
  for (int k = 0; k < 3; k++) {
    double ms = 0, mc[3] = {0}, Io[9] = {0}, mw, Iw[3];
    capsule_inertia(WHEEL_RHO, WHEEL_R, WHEEL_HH, &mw, Iw);
    add_geom_inertia(4 + k, mw, WHEEL_GPOS, m->wheel_gmat, Iw, &ms, mc, Io);
    finish_body(4 + k, ms, mc, Io);
  }
  {
    double ms = 0, mc[3] = {0}, Io[9] = {0};
    double mball = BALL_RHO * 4.0 / 3.0 * PI * BALL_R * BALL_R * BALL_R;
    double Ib[3] = {0.4 * mball * BALL_R * BALL_R, 0.4 * mball * BALL_R * BALL_R, 0.4 * mball * BALL_R * BALL_R};
    add_geom_inertia(7, mball, BALL_GPOS, I3, Ib, &ms, mc, Io);
    finish_body(7, ms, mc, Io);
    m->ball_mass = mball;
  }
  /* qpos0 */
  memset(m->qpos0, 0, sizeof m->qpos0);
  m->qpos0[2] = 0.24; m->qpos0[3] = 1;
  m->qpos0[12] = 0.26; m->qpos0[13] = 1;

  /* set0: invweight0 and meaninertia at qpos0 (mj_setConst) */
  double xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], xI[NB][9], xanc[3][3], xax[3][3];
  double scom[NB][3], cin[NB][36], cdof[NV][6], Mm[NV * NV];
  m->compiled = 1; /* kinematics uses the tables above */
  kinematics_all(m->qpos0, xpos, xquat, xmat, xipos, xI, xanc, xax);
  build_M(xmat, xpos, xipos, xI, xanc, xax, scom, cin, cdof, Mm);
  double tr = 0;
  for (int i = 0; i < NV; i++) tr += Mm[i * NV + i];
  m->meaninertia = tr / NV;
  double L[NV * NV];
  memcpy(L, Mm, sizeof L);
  chol(L, NV);
  for (int b = 1; b < NB; b++) {
    /* jacobian at body COM: jacp = cdof_lin + cdof_ang x (xipos - subtree_com[root]) */
    double jac[6][NV];
    memset(jac, 0, sizeof jac);
    for (int d = 0; d < NV; d++) {
      int in_chain = 0;
      if (d < 6) in_chain = (b >= 1 && b <= 6);
      else if (d < 9) in_chain = (b == 4 + (d - 6));
      else in_chain = (b == 7);
      if (!in_chain) continue;
      double off[3], w[3];
      v3sub(off, xipos[b], scom[body_root[b]]);
      v3cross(w, cdof[d], off);
      for (int i = 0; i < 3; i++) { jac[i][d] = cdof[d][3 + i] + w[i]; jac[3 + i][d] = cdof[d][i]; }
    }
    double A[6] = {0};
    for (int i = 0; i < 6; i++) {
      double x[NV];
      for (int d = 0; d < NV; d++) x[d] = jac[i][d];
      chol_solve(L, NV, x);
      double s = 0;
      for (int d = 0; d < NV; d++) s += jac[i][d] * x[d];
      A[i] = s;
    }
    m->invweight_tran[b] = (A[0] + A[1] + A[2]) / 3;
    m->invweight_rot[b] = (A[3] + A[4] + A[5]) / 3;
  }
}

void bbo_model_info(double* out) {
  compile_model();
  Model* m = &M_;
  /* [0..7] masses, [8..15] invweight_tran, [16..23] invweight_rot, [24] meaninertia,
   * [25..41] qpos0, [42..44] wheel0 ipos, [45..53] base inertia */
  for (int b = 0; b < NB; b++) { out[b] = m->mass[b]; out[8 + b] = m->invweight_tran[b]; out[16 + b] = m->invweight_rot[b]; }
  out[24] = m->meaninertia;
  for (int i = 0; i < NQ; i++) out[25 + i] = m->qpos0[i];
  for (int i = 0; i < 3; i++) out[42 + i] = m->ipos[4][i];
  for (int i = 0; i < 9; i++) out[45 + i] = m->inertia[1][i];
}

/* ---------------------------------------------------------- mj_kinematics */
static void kinematics_all(const double* qpos, double xpos[NB][3], double xquat[NB][4], double xmat[NB][9],
                           double xipos[NB][3], double xI[NB][9], double xanchor[3][3], double xaxis[3][3]) {
  Model* m = &M_;
  memset(xpos[0], 0, 3 * sizeof(double));
  xquat[0][0] = 1; xquat[0][1] = xquat[0][2] = xquat[0][3] = 0;
  q2mat(xmat[0], xquat[0]);
  for (int b = 1; b < NB; b++) {
    int p = body_parent[b];
    if (b == 1 || b == 7) { /* free joint */
      int a = (b == 1) ? 0 : 10;
      v3copy(xpos[b], qpos + a);
      memcpy(xquat[b], qpos + a + 3, 4 * sizeof(double));
      qnormalize(xquat[b]);
    } else {
      double t[3];
      m3v(t, xmat[p], m->body_pos[b]);
      v3add(xpos[b], xpos[p], t);
      qmul(xquat[b], xquat[p], m->body_quat[b]);
      if (b >= 4) { /* hinge */
        int k = b - 4;
        double R[9];
        q2mat(R, xquat[b]);
        m3v(t, R, HINGE_POS);
        v3add(xanchor[k], xpos[b], t);
        m3v(xaxis[k], R, m->jnt_axis);
        double ql[4];
        axisangle2quat(ql, m->jnt_axis, qpos[7 + k] - m->qpos0[7 + k]);
        qmul(xquat[b], xquat[b], ql);
        q2mat(R, xquat[b]);
        m3v(t, R, HINGE_POS);
        v3sub(xpos[b], xanchor[k], t);
      }
      qnormalize(xquat[b]);
    }
    q2mat(xmat[b], xquat[b]);
    double t[3], tmp[9];
    m3v(t, xmat[b], m->ipos[b]);
    v3add(xipos[b], xpos[b], t);
    m3mul(tmp, xmat[b], m->inertia[b]);
    m3mulT(xI[b], tmp, xmat[b]);
  }
}

/* body chain membership of dof d */
static int dof_in_chain(int d, int b) {
  if (d < 6) return b >= 1 && b <= 6;
  if (d < 9) return b == 4 + (d - 6);
  return b == 7;
}
static int dof_body(int d) { return d < 6 ? 1 : (d < 9 ? 4 + (d - 6) : 7); }

/* mj_comPos (subtree_com, cinert, cdof) + M = sum_b J_b' cinert_b J_b + armature */
static void build_M(const double xmat[NB][9], const double xpos[NB][3], const double xipos[NB][3],
                    const double xI[NB][9], const double xanchor[3][3], const double xaxis[3][3],
                    double subtree_com[NB][3], double cinert[NB][36], double cdof[NV][6], double* Mout) {
  Model* m = &M_;
  /* subtree com per tree root */
  for (int r = 0; r < NB; r++) { subtree_com[r][0] = subtree_com[r][1] = subtree_com[r][2] = 0; }
  double msum1 = 0;
  double c1[3] = {0, 0, 0};
  for (int b = 1; b <= 6; b++) { msum1 += m->mass[b]; for (int i = 0; i < 3; i++) c1[i] += m->mass[b] * xipos[b][i]; }
  for (int i = 0; i < 3; i++) c1[i] /= msum1;
  for (int b = 1; b <= 6; b++) v3copy(subtree_com[b], c1); /* per-body subtree com (only root's is used) */
  /* true per-body subtree com for the base is c1; store root values */
  v3copy(subtree_com[1], c1);
  v3copy(subtree_com[7], xipos[7]);
  /* cinert: spatial inertia at subtree_com[root], ordering (ang; lin) */
  for (int b = 1; b < NB; b++) {
    double* I6 = cinert[b];
    memset(I6, 0, 36 * sizeof(double));
    double r[3];
    v3sub(r, xipos[b], subtree_com[body_root[b]]);
    double mm = m->mass[b];
    double rx[9] = {0, -r[2], r[1], r[2], 0, -r[0], -r[1], r[0], 0};
    double rr = v3dot(r, r);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        I6[6 * i + j] = xI[b][3 * i + j] + mm * ((i == j ? rr : 0) - r[i] * r[j]);
        I6[6 * i + 3 + j] = mm * rx[3 * i + j];
        I6[6 * (3 + i) + j] = mm * rx[3 * j + i];
        I6[6 * (3 + i) + 3 + j] = (i == j) ? mm : 0;
      }
  }
  /* cdof */
  for (int d = 0; d < NV; d++) memset(cdof[d], 0, 6 * sizeof(double));
  for (int t = 0; t < 2; t++) {
    int b = t == 0 ? 1 : 7, da = t == 0 ? 0 : 9;
    for (int i = 0; i < 3; i++) cdof[da + i][3 + i] = 1;
    double off[3];
    v3sub(off, subtree_com[b], xpos[b]);
    for (int i = 0; i < 3; i++) {
      double ax[3] = {xmat[b][i], xmat[b][3 + i], xmat[b][6 + i]};
      v3copy(cdof[da + 3 + i], ax);
      v3cross(cdof[da + 3 + i] + 3, ax, off);
    }
  }
  for (int k = 0; k < 3; k++) {
    double off[3];
    v3sub(off, subtree_com[1], xanchor[k]);
    v3copy(cdof[6 + k], xaxis[k]);
    v3cross(cdof[6 + k] + 3, xaxis[k], off);
  }
  /* M */
  memset(Mout, 0, NV * NV * sizeof(double));
  for (int b = 1; b < NB; b++) {
    double IS[NV][6];
    for (int d = 0; d < NV; d++) {
      if (!dof_in_chain(d, b)) continue;
      for (int i = 0; i < 6; i++) {
        double s = 0;
        for (int j = 0; j < 6; j++) s += cinert[b][6 * i + j] * cdof[d][j];
        IS[d][i] = s;
      }
    }
    for (int d1 = 0; d1 < NV; d1++) {
      if (!dof_in_chain(d1, b)) continue;
      for (int d2 = 0; d2 < NV; d2++) {
        if (!dof_in_chain(d2, b)) continue;
        double s = 0;
        for (int i = 0; i < 6; i++) s += cdof[d1][i] * IS[d2][i];
        Mout[d1 * NV + d2] += s;
      }
    }
  }
  for (int k = 0; k < 3; k++) Mout[(6 + k) * NV + 6 + k] += HINGE_ARMATURE;
}

/* ------------------------------------------------------------ dense linalg */
static int chol(double* A, int n) { /* in place, lower */
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (s <= 0) return -1;
    double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 0;
}
static void chol_solve(const double* L, int n, double* x) {
  for (int i = 0; i < n; i++) {
    double s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

/* ---------------------------------------------------------- spatial algebra */
static void cross_motion(double* r, const double* v, const double* u) { /* v xm u */
  double t[6], a[3], b[3];
  v3cross(t, v, u);
  v3cross(a, v, u + 3);
  v3cross(b, v + 3, u);
  v3add(t + 3, a, b);
  memcpy(r, t, sizeof t);
}
static void cross_force(double* r, const double* v, const double* f) { /* v xf f */
  double t[6], a[3], b[3];
  v3cross(a, v, f);
  v3cross(b, v + 3, f + 3);
  v3add(t, a, b);
  v3cross(t + 3, v, f + 3);
  memcpy(r, t, sizeof t);
}
static void mul6(double* r, const double* I6, const double* v) {
  double t[6];
  for (int i = 0; i < 6; i++) { double s = 0; for (int j = 0; j < 6; j++) s += I6[6 * i + j] * v[j]; t[i] = s; }
  memcpy(r, t, sizeof t);
}

/* ------------------------------------------------------------- collision */
typedef struct {
  double dist, pos[3], frame[9];
  int body1, body2; /* jacdif = J(body2) - J(body1); normal points from geom1 (body1) to geom2 (body2) */
  double mu, fr[2];
} Contact;

/* mju_makeFrame: normalise x, default/orthogonalise y, z = x cross y */
static void make_frame(double* f) {
  v3normalize(f);
  if (v3norm(f + 3) < 0.5) {
    f[3] = f[4] = f[5] = 0;
    if (fabs(f[1]) < 0.5) f[4] = 1; else f[5] = 1;
  }
  double t[3];
  v3scl(t, f, v3dot(f, f + 3));
  v3sub(f + 3, f + 3, t);
  v3normalize(f + 3);
  v3cross(f + 6, f, f + 3);
}

/* closest point on triangle abc to p (Ericson, Real-Time Collision Detection 5.1.5) */
static void closest_pt_triangle(double* res, const double* p, const double* a, const double* b, const double* c) {
  double ab[3], ac[3], ap[3], bp[3], cp[3];
  v3sub(ab, b, a); v3sub(ac, c, a); v3sub(ap, p, a);
  double d1 = v3dot(ab, ap), d2 = v3dot(ac, ap);
  if (d1 <= 0 && d2 <= 0) { v3copy(res, a); return; }
  v3sub(bp, p, b);
  double d3 = v3dot(ab, bp), d4 = v3dot(ac, bp);
  if (d3 >= 0 && d4 <= d3) { v3copy(res, b); return; }
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) { double v = d1 / (d1 - d3); for (int i = 0; i < 3; i++) res[i] = a[i] + v * ab[i]; return; }
  v3sub(cp, p, c);
  double d5 = v3dot(ab, cp), d6 = v3dot(ac, cp);
  if (d6 >= 0 && d5 <= d6) { v3copy(res, c); return; }
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) { double w = d2 / (d2 - d6); for (int i = 0; i < 3; i++) res[i] = a[i] + w * ac[i]; return; }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int i = 0; i < 3; i++) res[i] = b[i] + w * (c[i] - b[i]);
    return;
  }
  double denom = 1.0 / (va + vb + vc), v = vb * denom, w = vc * denom;
  for (int i = 0; i < 3; i++) res[i] = a[i] + ab[i] * v + ac[i] * w;
}

/* Exact sphere (center c, radius r) vs triangular prism (top vertices T[3],
 * bottom plane z=zb) penetration: the minimum-translation result that the
 * convex penetration solver of mjc_ConvexHField converges to.
 * Returns 1 on contact with dist <= 0; fills dist, normal (prism -> sphere), pos. */
static int sphere_prism(const double* c, double r, double T[3][3], double zb, double* dist, double* n, double* pos) {
  double B[3][3];
  for (int i = 0; i < 3; i++) { B[i][0] = T[i][0]; B[i][1] = T[i][1]; B[i][2] = zb; }
  /* inside test: xy in triangle, above bottom, below top plane */
  double e1[3], e2[3], nt[3];
  v3sub(e1, T[1], T[0]); v3sub(e2, T[2], T[0]);
  v3cross(nt, e1, e2);
  if (nt[2] < 0) v3scl(nt, nt, -1);
  v3normalize(nt); /* top face outward normal (z >= 0) */
  /* 2D barycentric sign test */
  double area = (T[1][0] - T[0][0]) * (T[2][1] - T[0][1]) - (T[2][0] - T[0][0]) * (T[1][1] - T[0][1]);
  int inside_xy = 1;
  double sgn = area > 0 ? 1 : -1;
  double eout[3][3]; double edist[3];
  for (int i = 0; i < 3; i++) {
    const double* P = T[i]; const double* Q = T[(i + 1) % 3];
    double ex = Q[0] - P[0], ey = Q[1] - P[1];
    double cr = ex * (c[1] - P[1]) - ey * (c[0] - P[0]);
    if (cr * sgn < 0) inside_xy = 0;
    /* outward 2D normal of edge */
    double nx = ey * sgn, ny = -ex * sgn, nl = sqrt(nx * nx + ny * ny);
    eout[i][0] = nx / nl; eout[i][1] = ny / nl; eout[i][2] = 0;
    edist[i] = fabs(cr) / nl; /* distance of c to edge line (inside) */
  }
  double dtop = v3dot(nt, T[0]) - v3dot(nt, c); /* >0 when c below top plane */
  if (inside_xy && c[2] >= zb && dtop >= 0) {
    /* c inside prism: exit through nearest face */
    double best = dtop; double nb[3]; v3copy(nb, nt);
    if (c[2] - zb < best) { best = c[2] - zb; nb[0] = 0; nb[1] = 0; nb[2] = -1; }
    for (int i = 0; i < 3; i++) if (edist[i] < best) { best = edist[i]; v3copy(nb, eout[i]); }
    *dist = -best - r;
    v3copy(n, nb);
    for (int i = 0; i < 3; i++) pos[i] = c[i] - n[i] * (r + *dist / 2);
    return 1;
  }
  /* outside: closest point over the 5 faces (8 triangles) */
  double best = 1e300, q[3], qb[3];
  const double* tri[8][3] = {
      {T[0], T[1], T[2]}, {B[0], B[1], B[2]},
      {T[0], T[1], B[1]}, {T[0], B[1], B[0]},
      {T[1], T[2], B[2]}, {T[1], B[2], B[1]},
      {T[2], T[0], B[0]}, {T[2], B[0], B[2]}};
  for (int f = 0; f < 8; f++) {
    closest_pt_triangle(q, c, tri[f][0], tri[f][1], tri[f][2]);
    double dd[3]; v3sub(dd, c, q);
    double d2 = v3dot(dd, dd);
    if (d2 < best) { best = d2; v3copy(qb, q); }
  }
  double d = sqrt(best);
  if (d > r) return 0;
  if (d > 1e-12) { v3sub(n, c, qb); v3scl(n, n, 1.0 / d); }
  else { v3copy(n, nt); }
  *dist = d - r;
  for (int i = 0; i < 3; i++) pos[i] = c[i] - n[i] * (r + *dist / 2);
  return 1;
}


/* ---------------------------------------------- dynamic (contype) pairs
 * Besides the explicit ball-wheel pairs and ball-hfield, MuJoCo's broadphase
 * collides every other geom pair not filtered out (contype = conaffinity = 1
 * by default; ballbot.xml has no <exclude>; parent-child pairs are filtered,
 * the world body excepted):
 *   hfield x {tower cylinder, cam sticks (capsules), wheel capsules}
 *   ball   x {tower cylinder, cam sticks}
 * (ballast has contype 0; cam cone meshes are absent from the reference).
 * Contact geometry is exact: minimum-translation penetration by the
 * separating-axis theorem for capsule-prism (exact: prism face normals and
 * segment x edge axes) and cylinder-prism (face normals, cylinder axis,
 * axis x edges, vertex radials: exact except rim-edge contacts), closed form
 * for sphere-cylinder.  MuJoCo runs its convex penetration solver (MPR/EPA)
 * there, which agrees to its ccd tolerance. */
typedef struct { double c[3], a[3], hh, r; } Convex; /* capsule or cylinder: centre, unit axis, half-length, radius */

typedef struct { double V[6][3]; double pn[5][3], pd[5]; } Prism;

static void prism_build(Prism* P, double T[3][3], double zb) {
  for (int i = 0; i < 3; i++) {
    v3copy(P->V[i], T[i]);
    P->V[3 + i][0] = T[i][0]; P->V[3 + i][1] = T[i][1]; P->V[3 + i][2] = zb;
  }
  double e1[3], e2[3], nt[3];
  v3sub(e1, T[1], T[0]); v3sub(e2, T[2], T[0]);
  v3cross(nt, e1, e2);
  if (nt[2] < 0) v3scl(nt, nt, -1);
  v3normalize(nt);
  v3copy(P->pn[0], nt); P->pd[0] = v3dot(nt, T[0]);
  P->pn[1][0] = 0; P->pn[1][1] = 0; P->pn[1][2] = -1; P->pd[1] = -zb;
  double area = (T[1][0] - T[0][0]) * (T[2][1] - T[0][1]) - (T[2][0] - T[0][0]) * (T[1][1] - T[0][1]);
  double sgn = area > 0 ? 1 : -1;
  for (int i = 0; i < 3; i++) {
    const double* A = T[i]; const double* B = T[(i + 1) % 3];
    double ex = B[0] - A[0], ey = B[1] - A[1];
    double nx = ey * sgn, ny = -ex * sgn, nl = sqrt(nx * nx + ny * ny);
    P->pn[2 + i][0] = nx / nl; P->pn[2 + i][1] = ny / nl; P->pn[2 + i][2] = 0;
    P->pd[2 + i] = v3dot(P->pn[2 + i], A);
  }
}

static double prism_support(const Prism* P, const double* n) {
  double m = -1e300;
  for (int i = 0; i < 6; i++) { double d = v3dot(n, P->V[i]); if (d > m) m = d; }
  return m;
}

/* closest points of segments p0p1 and q0q1 (Ericson 5.1.9) */
static double seg_seg(const double* p0, const double* p1, const double* q0, const double* q1, double* cp, double* cq) {
  double d1[3], d2[3], r[3];
  v3sub(d1, p1, p0); v3sub(d2, q1, q0); v3sub(r, p0, q0);
  double a = v3dot(d1, d1), e = v3dot(d2, d2), f = v3dot(d2, r), s, t;
  if (a <= 1e-30 && e <= 1e-30) { s = t = 0; }
  else if (a <= 1e-30) { s = 0; t = f / e; t = t < 0 ? 0 : (t > 1 ? 1 : t); }
  else {
    double c = v3dot(d1, r);
    if (e <= 1e-30) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    else {
      double b = v3dot(d1, d2), den = a * e - b * b;
      s = den > 0 ? (b * f - c * e) / den : 0;
      s = s < 0 ? 0 : (s > 1 ? 1 : s);
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
      else if (t > 1) { t = 1; s = (b - c) / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    }
  }
  for (int i = 0; i < 3; i++) { cp[i] = p0[i] + s * d1[i]; cq[i] = q0[i] + t * d2[i]; }
  double d[3]; v3sub(d, cp, cq);
  return v3norm(d);
}

/* distance of segment p0p1 to triangle abc (0 if they intersect) */
static double seg_tri(const double* p0, const double* p1, const double* a, const double* b, const double* c,
                      double* cp, double* ct) {
  double e1[3], e2[3], n[3], d[3];
  v3sub(e1, b, a); v3sub(e2, c, a); v3cross(n, e1, e2); v3sub(d, p1, p0);
  double den = v3dot(n, d);
  if (fabs(den) > 1e-30) {
    double ap[3]; v3sub(ap, a, p0);
    double t = v3dot(n, ap) / den;
    if (t >= 0 && t <= 1) {
      double x[3]; for (int i = 0; i < 3; i++) x[i] = p0[i] + t * d[i];
      double q[3]; closest_pt_triangle(q, x, a, b, c);
      double dd[3]; v3sub(dd, x, q);
      if (v3dot(dd, dd) < 1e-28) { v3copy(cp, x); v3copy(ct, x); return 0; }
    }
  }
  double best = 1e300, q[3], dd[3], x1[3], x2[3];
  const double* ends[2] = {p0, p1};
  for (int k = 0; k < 2; k++) {
    closest_pt_triangle(q, ends[k], a, b, c);
    v3sub(dd, ends[k], q);
    double dist = v3norm(dd);
    if (dist < best) { best = dist; v3copy(cp, ends[k]); v3copy(ct, q); }
  }
  const double* E[3][2] = {{a, b}, {b, c}, {c, a}};
  for (int k = 0; k < 3; k++) {
    double dist = seg_seg(p0, p1, E[k][0], E[k][1], x1, x2);
    if (dist < best) { best = dist; v3copy(cp, x1); v3copy(ct, x2); }
  }
  return best;
}

static void convex_ends(const Convex* g, double* p0, double* p1) {
  for (int i = 0; i < 3; i++) { p0[i] = g->c[i] - g->hh * g->a[i]; p1[i] = g->c[i] + g->hh * g->a[i]; }
}

/* separating-axis depth along unit n for the segment of g (capsule core) vs prism:
 * how far the segment must move along +n to clear the prism */
static double seg_axis_depth(const Prism* P, const double* p0, const double* p1, const double* n) {
  double lo = fmin(v3dot(n, p0), v3dot(n, p1));
  return prism_support(P, n) - lo;
}

/* capsule vs prism; normal from prism to capsule */
static int capsule_prism(const Convex* g, const Prism* P, double* dist, double* n, double* pos) {
  double p0[3], p1[3];
  convex_ends(g, p0, p1);
  /* separated by more than r along a face normal: no contact */
  for (int f = 0; f < 5; f++)
    if (v3dot(P->pn[f], p0) - P->pd[f] >= g->r && v3dot(P->pn[f], p1) - P->pd[f] >= g->r) return 0;
  /* segment inside prism?  clip against the 5 half-spaces n.x <= d */
  double t0 = 0, t1 = 1, dir[3];
  v3sub(dir, p1, p0);
  int inter = 1;
  for (int f = 0; f < 5 && inter; f++) {
    double a0 = v3dot(P->pn[f], p0) - P->pd[f], ad = v3dot(P->pn[f], dir);
    if (fabs(ad) < 1e-30) { if (a0 > 0) inter = 0; continue; }
    double t = -a0 / ad;
    if (ad > 0) { if (t < t1) t1 = t; } else { if (t > t0) t0 = t; }
    if (t0 > t1) inter = 0;
  }
  if (!inter) {
    static const int tri[8][3] = {{0, 1, 2}, {3, 4, 5}, {0, 1, 4}, {0, 4, 3}, {1, 2, 5}, {1, 5, 4}, {2, 0, 3}, {2, 3, 5}};
    double best = 1e300, cp[3] = {0}, cq[3] = {0}, bp[3] = {0}, bq[3] = {0};
    for (int f = 0; f < 8; f++) {
      double d = seg_tri(p0, p1, P->V[tri[f][0]], P->V[tri[f][1]], P->V[tri[f][2]], cp, cq);
      if (d < best) { best = d; v3copy(bp, cp); v3copy(bq, cq); }
    }
    if (best >= g->r) return 0;
    if (best > 1e-12) { v3sub(n, bp, bq); v3scl(n, n, 1.0 / best); }
    else { v3copy(n, P->pn[0]); }
    *dist = best - g->r;
    for (int i = 0; i < 3; i++) pos[i] = bp[i] - n[i] * (g->r + *dist / 2);
    return 1;
  }
  /* intersecting: minimum over the separating-axis candidates */
  double axes[5 + 4][3];
  int na = 0;
  for (int f = 0; f < 5; f++) v3copy(axes[na++], P->pn[f]);
  double u[3]; v3copy(u, dir);
  double edges[4][3] = {{0, 0, 1}};
  for (int i = 0; i < 3; i++) v3sub(edges[1 + i], P->V[(i + 1) % 3], P->V[i]);
  for (int k = 0; k < 4; k++) {
    double x[3]; v3cross(x, u, edges[k]);
    if (v3norm(x) > 1e-12 * (v3norm(u) * v3norm(edges[k]) + 1e-30)) { v3normalize(x); v3copy(axes[na++], x); }
  }
  double bestd = 1e300, bn[3] = {0, 0, 1};
  for (int k = 0; k < na; k++)
    for (int sgn = -1; sgn <= 1; sgn += 2) {
      double ax[3]; v3scl(ax, axes[k], sgn);
      double d = seg_axis_depth(P, p0, p1, ax);
      if (d < bestd) { bestd = d; v3copy(bn, ax); }
    }
  v3copy(n, bn);
  *dist = -bestd - g->r;
  /* deepest segment point along -n; when the segment is (nearly) normal to
   * -n the deepest set is the clipped part [t0, t1] of the segment: take the
   * point of it nearest the prism centroid */
  double e0 = v3dot(n, p0), e1 = v3dot(n, p1), xd[3];
  if (fabs(e0 - e1) < 1e-12) {
    double cen[3] = {0, 0, 0}, dd = v3dot(dir, dir);
    for (int v = 0; v < 6; v++) for (int i = 0; i < 3; i++) cen[i] += P->V[v][i] / 6;
    double cp0[3]; v3sub(cp0, cen, p0);
    double t = dd > 0 ? v3dot(cp0, dir) / dd : 0;
    t = t < t0 ? t0 : (t > t1 ? t1 : t);
    for (int i = 0; i < 3; i++) xd[i] = p0[i] + t * dir[i];
  } else {
    v3copy(xd, e0 < e1 ? p0 : p1);
  }
  for (int i = 0; i < 3; i++) pos[i] = xd[i] - n[i] * (g->r + *dist / 2);
  return 1;
}

static double cyl_support(const Convex* g, const double* n) {
  double na = v3dot(n, g->a);
  double rad = 1 - na * na;
  return v3dot(n, g->c) + g->hh * fabs(na) + g->r * sqrt(rad > 0 ? rad : 0);
}

/* cylinder vs prism; normal from prism to cylinder */
static int cylinder_prism(const Convex* g, const Prism* P, double* dist, double* n, double* pos) {
  double axes[5 + 1 + 4 + 6][3];
  int na = 0;
  for (int f = 0; f < 5; f++) v3copy(axes[na++], P->pn[f]);
  v3copy(axes[na++], g->a);
  double edges[4][3] = {{0, 0, 1}};
  for (int i = 0; i < 3; i++) v3sub(edges[1 + i], P->V[(i + 1) % 3], P->V[i]);
  for (int k = 0; k < 4; k++) {
    double x[3]; v3cross(x, g->a, edges[k]);
    if (v3norm(x) > 1e-12 * (v3norm(edges[k]) + 1e-30)) { v3normalize(x); v3copy(axes[na++], x); }
  }
  for (int i = 0; i < 6; i++) {
    double d[3], x[3]; v3sub(d, P->V[i], g->c);
    double t = v3dot(d, g->a);
    for (int k = 0; k < 3; k++) x[k] = d[k] - t * g->a[k];
    if (v3norm(x) > 1e-12) { v3normalize(x); v3copy(axes[na++], x); }
  }
  double bestd = 1e300, bn[3] = {0, 0, 1};
  for (int k = 0; k < na; k++)
    for (int sgn = -1; sgn <= 1; sgn += 2) {
      double ax[3], mx[3]; v3scl(ax, axes[k], sgn);
      v3scl(mx, ax, -1);
      double d = prism_support(P, ax) + cyl_support(g, mx); /* = max_P ax.y - min_C ax.x */
      if (d <= 0) return 0; /* separating axis */
      if (d < bestd) { bestd = d; v3copy(bn, ax); }
    }
  v3copy(n, bn);
  *dist = -bestd;
  /* deepest cylinder point along -n; in the degenerate directions (n normal
   * to the axis: a generator line; n along the axis: a cap disk) the point of
   * that set nearest the prism centroid */
  double na2 = v3dot(n, g->a), s[3], rad[3], cen[3] = {0, 0, 0}, dc[3];
  for (int v = 0; v < 6; v++) for (int k = 0; k < 3; k++) cen[k] += P->V[v][k] / 6;
  v3sub(dc, cen, g->c);
  for (int k = 0; k < 3; k++) rad[k] = n[k] - na2 * g->a[k];
  double rl = v3norm(rad);
  double along;
  if (fabs(na2) > 1e-9) along = na2 > 0 ? -g->hh : g->hh;
  else { along = v3dot(dc, g->a); along = along > g->hh ? g->hh : (along < -g->hh ? -g->hh : along); }
  for (int k = 0; k < 3; k++) s[k] = g->c[k] + along * g->a[k];
  if (rl > 1e-9) {
    for (int k = 0; k < 3; k++) s[k] -= g->r * rad[k] / rl;
  } else {
    double pr[3], t = v3dot(dc, g->a);
    for (int k = 0; k < 3; k++) pr[k] = dc[k] - t * g->a[k];
    double pl = v3norm(pr);
    if (pl > g->r) v3scl(pr, pr, g->r / pl);
    for (int k = 0; k < 3; k++) s[k] += pr[k];
  }
  for (int k = 0; k < 3; k++) pos[k] = s[k] - n[k] * (*dist / 2);
  return 1;
}

/* sphere (geom1) vs cylinder (geom2): normal from sphere to cylinder */
static int sphere_cylinder(const double* c, double r, const Convex* g, double* dist, double* n, double* pos) {
  double d[3]; v3sub(d, c, g->c);
  double z = v3dot(d, g->a), rv[3];
  for (int k = 0; k < 3; k++) rv[k] = d[k] - z * g->a[k];
  double rho = v3norm(rv), u[3] = {0, 0, 0};
  if (rho > 1e-12) v3scl(u, rv, 1.0 / rho);
  int inside = fabs(z) <= g->hh && rho <= g->r;
  double q[3];
  if (!inside) {
    double zc = z > g->hh ? g->hh : (z < -g->hh ? -g->hh : z);
    double rc = rho > g->r ? g->r : rho;
    for (int k = 0; k < 3; k++) q[k] = g->c[k] + zc * g->a[k] + rc * u[k];
    double dq[3]; v3sub(dq, q, c);
    double dd = v3norm(dq);
    if (dd >= r) return 0;
    *dist = dd - r;
    if (dd > 1e-12) v3scl(n, dq, 1.0 / dd); else v3copy(n, g->a);
  } else {
    double ds = g->r - rho, dc = g->hh - fabs(z);
    if (ds < dc) { /* exit through the side: the cylinder surface lies outward along u */
      for (int k = 0; k < 3; k++) n[k] = -u[k];
      *dist = -ds - r;
    } else {
      double sg = z >= 0 ? 1 : -1;
      for (int k = 0; k < 3; k++) n[k] = -sg * g->a[k];
      *dist = -dc - r;
    }
  }
  for (int k = 0; k < 3; k++) pos[k] = c[k] + n[k] * (r + *dist / 2);
  return 1;
}

/* world poses of the convex geoms of the base tree: 0 tower, 1-2 cam sticks, 3-5 wheels */
static void body_geoms(const double xpos[NB][3], const double xmat[NB][9], Convex g[6], int cyl[6], int body[6]) {
  Model* m = &M_;
  double t[3];
  /* tower_collision: cylinder r .11 hh .14 at (0,0,0.2) of base (ballbot.xml:41) */
  const double tower_c[3] = {0, 0, 0.2};
  m3v(t, xmat[1], tower_c);
  v3add(g[0].c, xpos[1], t);
  g[0].a[0] = xmat[1][2]; g[0].a[1] = xmat[1][5]; g[0].a[2] = xmat[1][8];
  g[0].hh = 0.14; g[0].r = 0.11; cyl[0] = 1; body[0] = 1;
  /* cam_k_stick: capsule fromto (0,0,0)->(-+0.2,0,0), r .01 (ballbot.xml:46,52) */
  for (int k = 0; k < 2; k++) {
    int b = 2 + k;
    double lc[3] = {k == 0 ? -0.1 : 0.1, 0, 0};
    m3v(t, xmat[b], lc);
    v3add(g[1 + k].c, xpos[b], t);
    g[1 + k].a[0] = xmat[b][0]; g[1 + k].a[1] = xmat[b][3]; g[1 + k].a[2] = xmat[b][6];
    g[1 + k].hh = 0.1; g[1 + k].r = 0.01; cyl[1 + k] = 0; body[1 + k] = b;
  }
  /* wheel_mesh_k: capsule r .025 hh .02 (ballbot.xml:57,62,68) */
  for (int k = 0; k < 3; k++) {
    int b = 4 + k;
    double gm[9];
    m3v(t, xmat[b], WHEEL_GPOS);
    v3add(g[3 + k].c, xpos[b], t);
    m3mul(gm, xmat[b], m->wheel_gmat);
    g[3 + k].a[0] = gm[2]; g[3 + k].a[1] = gm[5]; g[3 + k].a[2] = gm[8];
    g[3 + k].hh = WHEEL_HH; g[3 + k].r = WHEEL_R; cyl[3 + k] = 0; body[3 + k] = b;
  }
}

static int collide(const double xpos[NB][3], const double xmat[NB][9], const float* hf, double size_z,
                   Contact* con, int* nground_out, int* nbody_out, int* overflow) {
  Model* m = &M_;
  int n = 0;
  double c[3], t[3];
  m3v(t, xmat[7], BALL_GPOS);
  v3add(c, xpos[7], t);
  /* explicit pairs ballbot.xml:90-92: the_ball x wheel_mesh_k, condim 3,
   * friction (0.001, 1.0).  mjraw_SphereCapsule (+ mujoco_fix.patch). */
  for (int k = 0; k < 3; k++) {
    int b = 4 + k;
    double gp[3], gm[9];
    m3v(t, xmat[b], WHEEL_GPOS);
    v3add(gp, xpos[b], t);
    m3mul(gm, xmat[b], m->wheel_gmat);
    double axis[3] = {gm[2], gm[5], gm[8]};
    double vec[3];
    v3sub(vec, c, gp);
    double x = v3dot(axis, vec);
    if (x > WHEEL_HH) x = WHEEL_HH;
    if (x < -WHEEL_HH) x = -WHEEL_HH;
    double near[3];
    for (int i = 0; i < 3; i++) near[i] = gp[i] + axis[i] * x;
    double dif[3];
    v3sub(dif, near, c);
    double cdist = v3norm(dif);
    double dist = cdist - BALL_R - WHEEL_R;
    if (dist > 0) continue;
    Contact* cc = &con[n++];
    memset(cc, 0, sizeof *cc);
    cc->dist = dist;
    if (cdist > 0) v3scl(cc->frame, dif, 1.0 / cdist);
    else { cc->frame[0] = 1; }
    v3copy(cc->frame + 3, axis); /* mujoco_fix.patch:15 */
    make_frame(cc->frame);
    for (int i = 0; i < 3; i++) cc->pos[i] = c[i] + cc->frame[i] * (BALL_R + dist / 2);
    cc->body1 = 7; cc->body2 = b;
    cc->fr[0] = 0.001; cc->fr[1] = 1.0;
  }
  int nground = 0;
  *overflow = 0;
  if (hf) {
    /* mjc_ConvexHField: hfield geom at origin, identity frame (ballbot.xml:35) */
    double xmin = c[0] - BALL_R, xmax = c[0] + BALL_R, ymin = c[1] - BALL_R, ymax = c[1] + BALL_R;
    double zmin = c[2] - BALL_R, zmax = c[2] + BALL_R;
    const double sx = HF_SIZE[0], sy = HF_SIZE[1], zb = HF_SIZE[3];
    const int nrow = BBO_HF_N, ncol = BBO_HF_N;
    if (!(xmin > sx || xmax < -sx || ymin > sy || ymax < -sy || zmin > size_z || zmax < -zb)) {
      int cmin = (int)floor((xmin + sx) / (2 * sx) * (ncol - 1));
      int cmax = (int)ceil((xmax + sx) / (2 * sx) * (ncol - 1));
      int rmin = (int)floor((ymin + sy) / (2 * sy) * (nrow - 1));
      int rmax = (int)ceil((ymax + sy) / (2 * sy) * (nrow - 1));
      if (cmin < 0) cmin = 0;
      if (cmax > ncol - 1) cmax = ncol - 1;
      if (rmin < 0) rmin = 0;
      if (rmax > nrow - 1) rmax = nrow - 1;
      double dx = 2 * sx / (ncol - 1), dy = 2 * sy / (nrow - 1);
      for (int r = rmin; r < rmax; r++) {
        double win[3][3] = {{0}};
        int nvert = 0;
        for (int cc = cmin; cc <= cmax; cc++) {
          for (int i = 0; i < 2; i++) {
            win[0][0] = win[1][0]; win[0][1] = win[1][1]; win[0][2] = win[1][2];
            win[1][0] = win[2][0]; win[1][1] = win[2][1]; win[1][2] = win[2][2];
            win[2][0] = dx * cc - sx;
            win[2][1] = dy * (r + i) - sy;
            win[2][2] = (double)hf[(r + i) * ncol + cc] * size_z;
            nvert++;
            if (nvert <= 2) continue;
            if (win[0][2] < zmin && win[1][2] < zmin && win[2][2] < zmin) continue;
            double dist, nn[3], pos[3];
            if (!sphere_prism(c, BALL_R, win, -zb, &dist, nn, pos)) continue;
            if (nground >= BBO_MAXGROUND) { *overflow = 1; continue; }
            Contact* g = &con[n++];
            memset(g, 0, sizeof *g);
            g->dist = dist;
            v3copy(g->frame, nn);
            make_frame(g->frame);
            v3copy(g->pos, pos);
            g->body1 = 0; g->body2 = 7;
            g->fr[0] = 1.0; g->fr[1] = 1.0; /* max(geom friction) = (1,1,0.005,..) */
            nground++;
          }
        }
      }
    }
  }
  *nground_out = nground;

  /* dynamic pairs with the base-tree geoms (see body_geoms) */
  Convex bg[6];
  int cyl[6], bbody[6];
  body_geoms(xpos, xmat, bg, cyl, bbody);
  int nbody = 0;
  /* ball (geom1, sphere) x tower (cylinder) / cam sticks (capsules, patched frame) */
  for (int k = 0; k < 3; k++) {
    double dist, nn[3], pos[3];
    int hit;
    if (cyl[k]) {
      hit = sphere_cylinder(c, BALL_R, &bg[k], &dist, nn, pos);
    } else {
      double p0[3], p1[3], cp[3], cq[3];
      convex_ends(&bg[k], p0, p1);
      double d = seg_seg(c, c, p0, p1, cp, cq);
      dist = d - BALL_R - bg[k].r;
      hit = dist <= 0;
      if (hit) {
        if (d > 0) { v3sub(nn, cq, c); v3scl(nn, nn, 1.0 / d); } else { nn[0] = 1; nn[1] = nn[2] = 0; }
        for (int i = 0; i < 3; i++) pos[i] = c[i] + nn[i] * (BALL_R + dist / 2);
      }
    }
    if (!hit) continue;
    Contact* b = &con[n++];
    memset(b, 0, sizeof *b);
    b->dist = dist;
    v3copy(b->frame, nn);
    if (!cyl[k]) v3copy(b->frame + 3, bg[k].a); /* mujoco_fix.patch: capsule axis as first tangent */
    make_frame(b->frame);
    v3copy(b->pos, pos);
    b->body1 = 7; b->body2 = bbody[k];
    b->fr[0] = 1.0; b->fr[1] = 1.0;
    nbody++;
  }
  /* hfield (geom1) x convex geom (mjc_ConvexHField): prisms under the geom's AABB */
  if (hf) {
    const double sx = HF_SIZE[0], sy = HF_SIZE[1], zb = HF_SIZE[3];
    const int nrow = BBO_HF_N, ncol = BBO_HF_N;
    const double dx = 2 * sx / (ncol - 1), dy = 2 * sy / (nrow - 1);
    for (int k = 0; k < 6; k++) {
      const Convex* g = &bg[k];
      int npair = 0; /* mjc_ConvexHField keeps the pair's first mjMAXCONPAIR contacts */
      double lo[3], hi[3];
      for (int i = 0; i < 3; i++) {
        double ai = fabs(g->a[i]);
        double ext = cyl[k] ? g->hh * ai + g->r * sqrt(fmax(0.0, 1 - ai * ai)) : g->hh * ai + g->r;
        lo[i] = g->c[i] - ext; hi[i] = g->c[i] + ext;
      }
      if (lo[0] > sx || hi[0] < -sx || lo[1] > sy || hi[1] < -sy || lo[2] > size_z || hi[2] < -zb) continue;
      int cmin = (int)floor((lo[0] + sx) / (2 * sx) * (ncol - 1));
      int cmax = (int)ceil((hi[0] + sx) / (2 * sx) * (ncol - 1));
      int rmin = (int)floor((lo[1] + sy) / (2 * sy) * (nrow - 1));
      int rmax = (int)ceil((hi[1] + sy) / (2 * sy) * (nrow - 1));
      if (cmin < 0) cmin = 0;
      if (cmax > ncol - 1) cmax = ncol - 1;
      if (rmin < 0) rmin = 0;
      if (rmax > nrow - 1) rmax = nrow - 1;
      for (int r = rmin; r < rmax; r++) {
        double win[3][3] = {{0}};
        int nvert = 0;
        for (int cc = cmin; cc <= cmax; cc++) {
          for (int i = 0; i < 2; i++) {
            win[0][0] = win[1][0]; win[0][1] = win[1][1]; win[0][2] = win[1][2];
            win[1][0] = win[2][0]; win[1][1] = win[2][1]; win[1][2] = win[2][2];
            win[2][0] = dx * cc - sx;
            win[2][1] = dy * (r + i) - sy;
            win[2][2] = (double)hf[(r + i) * ncol + cc] * size_z;
            nvert++;
            if (nvert <= 2) continue;
            if (win[0][2] < lo[2] && win[1][2] < lo[2] && win[2][2] < lo[2]) continue;
            Prism P;
            prism_build(&P, win, -zb);
            double dist, nn[3], pos[3];
            int hit = cyl[k] ? cylinder_prism(g, &P, &dist, nn, pos) : capsule_prism(g, &P, &dist, nn, pos);
            if (!hit) continue;
            if (npair >= BBO_MAXPAIR) { *overflow |= 2; continue; } /* MuJoCo drops these too */
            npair++;
            Contact* b = &con[n++];
            memset(b, 0, sizeof *b);
            b->dist = dist;
            v3copy(b->frame, nn);
            make_frame(b->frame);
            v3copy(b->pos, pos);
            b->body1 = 0; b->body2 = bbody[k];
            b->fr[0] = 1.0; b->fr[1] = 1.0;
            nbody++;
          }
        }
      }
    }
  }
  *nbody_out = nbody;
  return n;
}

/* ----------------------------------------------------------- constraints */
static double impedance(double pos) { /* getImpedance with solimp (0.9,0.95,0.001,0.5,2) */
  const double s0 = 0.9, s1 = 0.95, w = 0.001, mid = 0.5, pw = 2;
  double x = pos / w;
  if (x < 0) x = -x;
  if (x >= 1 || x <= 0) return x >= 1 ? s1 : s0;
  double y;
  if (x <= mid) y = pow(x, pw) / pow(mid, pw - 1);
  else y = 1 - pow(1 - x, pw) / pow(1 - mid, pw - 1);
  return s0 + y * (s1 - s0);
}

typedef struct {
  int nc;
  double J[BBO_MAXCON * 3][NV];
  double aref[BBO_MAXCON * 3], D[BBO_MAXCON * 3];
  double mu[BBO_MAXCON], fr[BBO_MAXCON][2];
} Efc;

/* contact cost/force/hessian for one elliptic condim-3 contact (mj_constraintUpdate) */
static double cone_eval(const double* jar, double mu, const double* fr, const double* D, double* force, double H[3][3]) {
  double U0 = jar[0] * mu, U1 = jar[1] * fr[0], U2 = jar[2] * fr[1];
  double N = U0, T = sqrt(U1 * U1 + U2 * U2);
  double cost = 0;
  if (H) memset(H, 0, 9 * sizeof(double));
  if (N >= mu * T || (T <= 0 && N >= 0)) { /* top zone */
    force[0] = force[1] = force[2] = 0;
  } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) { /* bottom zone */
    for (int j = 0; j < 3; j++) { force[j] = -D[j] * jar[j]; cost += 0.5 * D[j] * jar[j] * jar[j]; if (H) H[j][j] = D[j]; }
  } else { /* middle zone */
    double Dm = D[0] / (mu * mu * (1 + mu * mu));
    double g = N - mu * T;
    cost = 0.5 * Dm * g * g;
    double Ut[2] = {U1, U2};
    double grad[3] = {mu, -mu * fr[0] * U1 / T, -mu * fr[1] * U2 / T};
    for (int j = 0; j < 3; j++) force[j] = -Dm * g * grad[j];
    if (H) {
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) H[a][b] = Dm * grad[a] * grad[b];
      for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++) {
          double h2 = -mu * fr[a] * fr[b] * ((a == b ? 1.0 / T : 0) - Ut[a] * Ut[b] / (T * T * T));
          H[1 + a][1 + b] += Dm * g * h2;
        }
    }
  }
  return cost;
}

static double total_cost(const Efc* e, const double* jar, double* force, double* Hrows /*nullable*/) {
  double cost = 0;
  for (int c = 0; c < e->nc; c++) {
    double H[3][3];
    cost += cone_eval(jar + 3 * c, e->mu[c], e->fr[c], e->D + 3 * c, force + 3 * c, Hrows ? H : NULL);
    if (Hrows) memcpy(Hrows + 9 * c, H, sizeof H);
  }
  return cost;
}

/* ------------------------------------------------------------------------
 * mj_solNewton: MuJoCo's primal solver with flg_Newton (mj_solPrimal,
 * PrimalUpdateConstraint/-Gradient, PrimalPrepare/-Eval/-Search in
 * engine_solver.c at the commit the reference pins, 99490163, Readme.md:101-103).
 * MuJoCo is not in /root/reference, so this restatement of its published source
 * is PARITY UNPINNED [MJ].  The GPU kernel keeps its own line search (bb_solve.h
 * LineSearch); tests/ hold the two to a stated tolerance, not to bit equality.
 *
 *   cost(a)   = 0.5 (a - a0)' M (a - a0) + sum_c phi_c(J_c a - aref_c)   (Gauss + elliptic cones)
 *   iteration H = M + sum_c J_c' C_c J_c (cone Hessians, incl. the middle zone's
 *             cross terms); search s = -H^-1 grad; alpha = PrimalSearch(s); a += alpha s;
 *             recompute cost and gradient; stop when alpha == 0, or
 *             scale (oldcost - cost) < tolerance, or scale |grad| < tolerance
 *             (scale = 1 / (meaninertia max(1, nv)))
 *   search    MuJoCo's PrimalSearch: p1 = one Newton step from alpha 0 (kept only if it
 *             lowers the cost); converged when |phi'(alpha)| < gtol with
 *             gtol = tolerance ls_tolerance |s| / scale; else Newton steps in the
 *             descent direction until phi' changes sign (the bracket [p2, p1]), then
 *             rounds of three candidates -- the Newton points of both bracket ends
 *             and the midpoint -- returning the cheapest converged candidate, or
 *             moving each bracket end to a candidate with a same-signed, smaller |phi'|;
 *             every evaluation counts against ls_iterations.
 * ------------------------------------------------------------------------ */

/* One contact along the search line (PrimalPrepare for an elliptic cone): the cone
 * variables U(alpha) = u0 + alpha du (U0 = mu jar0, U1 = f1 jar1, U2 = f2 jar2, as
 * cone_eval) and the bottom zone's quadratic in alpha (c0, b0, b1). */
typedef struct { double u0[3], du[3], mu, Dm, b0, b1, c0, vv; } ConeLine;

static void cone_line_prep(ConeLine* t, const double* j0, const double* x, double mu, double f1, double f2,
                           const double* D) {
  t->mu = mu;
  t->Dm = D[0] / (mu * mu * (1 + mu * mu));
  t->u0[0] = mu * j0[0]; t->u0[1] = f1 * j0[1]; t->u0[2] = f2 * j0[2];
  t->du[0] = mu * x[0]; t->du[1] = f1 * x[1]; t->du[2] = f2 * x[2];
  t->b0 = D[0] * j0[0] * x[0] + D[1] * j0[1] * x[1] + D[2] * j0[2] * x[2];
  t->b1 = D[0] * x[0] * x[0] + D[1] * x[1] * x[1] + D[2] * x[2] * x[2];
  t->c0 = 0.5 * (D[0] * j0[0] * j0[0] + D[1] * j0[1] * j0[1] + D[2] * j0[2] * j0[2]);
  t->vv = t->du[1] * t->du[1] + t->du[2] * t->du[2];
}

/* the contact's cost phi_c(alpha) and its first two derivatives (PrimalEval), by
 * cone_eval's zones: top (N >= mu T) nothing; bottom (mu N + T <= 0) the three
 * rows' quadratics; middle 0.5 Dm (N - mu T)^2 with T(alpha) a hyperbola */
static void cone_line_eval(const ConeLine* t, double alpha, double* cost, double* d0, double* d1) {
  const double N = t->u0[0] + alpha * t->du[0], U1 = t->u0[1] + alpha * t->du[1], U2 = t->u0[2] + alpha * t->du[2];
  const double T = sqrt(U1 * U1 + U2 * U2), mu = t->mu;
  if (N >= mu * T) return;
  if (mu * N + T <= 0) {
    *cost += t->c0 + alpha * (t->b0 + 0.5 * alpha * t->b1);
    *d0 += t->b0 + alpha * t->b1;
    *d1 += t->b1;
    return;
  }
  /* middle zone: T > 0 here (T = 0 would need N < 0 and mu N > 0) */
  const double g = N - mu * T;
  const double tp = (U1 * t->du[1] + U2 * t->du[2]) / T;
  const double tpp = (t->vv - tp * tp) / T;
  const double gp = t->du[0] - mu * tp;
  *cost += 0.5 * t->Dm * g * g;
  *d0 += t->Dm * g * gp;
  *d1 += t->Dm * (gp * gp - mu * g * tpp);
}

/* a point of the line search (mjPrimalPnt): alpha, cost, phi', phi'' */
typedef struct { double alpha, cost, d0, d1; } PrimalPnt;

typedef struct {
  int nc, evals;
  double q0, q1, q2;  /* Gauss cost on the line: q0 + alpha q1 + alpha^2 q2 */
  const ConeLine* cl;
} PrimalLine;

static void primal_eval(PrimalLine* L, PrimalPnt* p) {
  const double a = p->alpha;
  double cost = L->q0 + a * (L->q1 + a * L->q2), d0 = L->q1 + 2 * a * L->q2, d1 = 2 * L->q2;
  for (int c = 0; c < L->nc; c++) cone_line_eval(&L->cl[c], a, &cost, &d0, &d1);
  p->cost = cost; p->d0 = d0; p->d1 = d1;
  L->evals++;
}

/* updateBracket: move bracket end p to a candidate on its side of the minimum
 * (same sign of phi') with a smaller |phi'|; then its Newton point pnext */
static int update_bracket(PrimalLine* L, PrimalPnt* p, PrimalPnt* const cand[3], PrimalPnt* pnext) {
  int flag = 0;
  for (int i = 0; i < 3; i++) {
    if (p->d0 < 0 && cand[i]->d0 < 0 && p->d0 < cand[i]->d0) { *p = *cand[i]; flag = 1; }
    else if (p->d0 > 0 && cand[i]->d0 > 0 && p->d0 > cand[i]->d0) { *p = *cand[i]; flag = 2; }
  }
  if (flag) {
    pnext->alpha = p->alpha - p->d0 / p->d1;
    primal_eval(L, pnext);
  }
  return flag;
}

/* PrimalSearch -> alpha (0: no improvement) */
static double primal_search(PrimalLine* L, double snorm, double scale) {
  if (snorm < MJMINVAL) return 0;
  const double gtol = g_tol * g_lstol * snorm / scale;
  PrimalPnt p0, p1, p2, pmid, p1next, p2next;
  L->evals = 0;
  p0.alpha = 0;
  primal_eval(L, &p0);
  p1.alpha = p0.alpha - p0.d0 / p0.d1;  /* always attempt one Newton step */
  primal_eval(L, &p1);
  if (p0.cost < p1.cost) p1 = p0;
  if (fabs(p1.d0) < gtol) return p1.alpha;  /* initial convergence (alpha 0: no improvement) */
  const double dir = p1.d0 < 0 ? 1 : -1;
  int p2update = 0;
  while (p1.d0 * dir <= -gtol && L->evals < g_lsmax) {  /* one-sided: Newton steps until phi' changes sign */
    p2 = p1;
    p2update = 1;
    p1.alpha -= p1.d0 / p1.d1;
    primal_eval(L, &p1);
    if (fabs(p1.d0) < gtol) return p1.alpha;
  }
  if (L->evals >= g_lsmax || !p2update) return p1.alpha;  /* could not bracket */
  p1next.alpha = p1.alpha - p1.d0 / p1.d1;
  primal_eval(L, &p1next);
  p2next.alpha = p2.alpha - p2.d0 / p2.d1;
  primal_eval(L, &p2next);
  while (L->evals < g_lsmax) {  /* bracketed */
    pmid.alpha = 0.5 * (p1.alpha + p2.alpha);
    primal_eval(L, &pmid);
    PrimalPnt* const cand[3] = {&p1next, &p2next, &pmid};
    int best = -1;
    double bestcost = 0;
    for (int i = 0; i < 3; i++)
      if (fabs(cand[i]->d0) < gtol && (best < 0 || cand[i]->cost < bestcost)) { bestcost = cand[i]->cost; best = i; }
    if (best >= 0) return cand[best]->alpha;
    /* both ends update from the same three candidates (copies: p1's update must not move p2's) */
    PrimalPnt c0 = p1next, c1 = p2next, c2 = pmid;
    PrimalPnt* const cc[3] = {&c0, &c1, &c2};
    const int b1 = update_bracket(L, &p1, cc, &p1next);
    const int b2 = update_bracket(L, &p2, cc, &p2next);
    if (!b1 && !b2) return pmid.alpha;  /* numerical accuracy reached: the midpoint */
  }
  /* out of evaluations: the better bracket end, if it improves on alpha 0 */
  if (p1.cost <= p2.cost && p1.cost < p0.cost) return p1.alpha;
  if (p2.cost <= p1.cost && p2.cost < p0.cost) return p2.alpha;
  return 0;
}

/* the solver's state at qacc a (PrimalUpdateConstraint + PrimalUpdateGradient):
 * jar = J a - aref, cone forces and Hessians, cost = Gauss + constraint, grad */
typedef struct {
  double jar[BBO_MAXCON * 3], force[BBO_MAXCON * 3], Hc[BBO_MAXCON * 9];
  double dq[NV], Mdq[NV], grad[NV], cost;
} PrimalState;

static void primal_update(const Efc* e, const double* Mm, const double* a0, const double* a, PrimalState* S) {
  const int nr = 3 * e->nc;
  for (int r = 0; r < nr; r++) { double s = -e->aref[r]; for (int d = 0; d < NV; d++) s += e->J[r][d] * a[d]; S->jar[r] = s; }
  const double ccost = total_cost(e, S->jar, S->force, S->Hc);
  double gauss = 0;
  for (int d = 0; d < NV; d++) S->dq[d] = a[d] - a0[d];
  for (int i = 0; i < NV; i++) {
    double s = 0;
    for (int j = 0; j < NV; j++) s += Mm[i * NV + j] * S->dq[j];
    S->Mdq[i] = s;
    gauss += 0.5 * S->dq[i] * s;
  }
  for (int i = 0; i < NV; i++) {
    double s = S->Mdq[i];
    for (int r = 0; r < nr; r++) s -= e->J[r][i] * S->force[r];
    S->grad[i] = s;
  }
  S->cost = gauss + ccost;
}

/* Newton solve of min 0.5(a-a0)'M(a-a0) + s(Ja - aref) from a (the warm start) */
static int newton(const Efc* e, const double* Mm, const double* a0, double* a, double scale) {
  const int nr = 3 * e->nc;
  static __thread PrimalState S;
  static __thread ConeLine cl[BBO_MAXCON];
  primal_update(e, Mm, a0, a, &S);
  int it;
  for (it = 0; it < g_maxiter; it++) {
    if (g_flags & 256) {
      double gn = 0;
      for (int i = 0; i < NV; i++) gn += S.grad[i] * S.grad[i];
      fprintf(stderr, "it %d cost %.17g grad %.3e\n", it, scale * S.cost, scale * sqrt(gn));
    }
    double H[NV * NV];
    memcpy(H, Mm, sizeof H);
    for (int c = 0; c < e->nc; c++) {
      const double* C = S.Hc + 9 * c;
      for (int p = 0; p < 3; p++)
        for (int q = 0; q < 3; q++) {
          double w = C[3 * p + q];
          if (w == 0) continue;
          for (int i = 0; i < NV; i++) {
            double ji = e->J[3 * c + p][i];
            if (ji == 0) continue;
            for (int j = 0; j < NV; j++) H[i * NV + j] += ji * w * e->J[3 * c + q][j];
          }
        }
    }
    if (chol(H, NV)) break;
    double s[NV], snorm = 0;
    for (int i = 0; i < NV; i++) s[i] = -S.grad[i];
    chol_solve(H, NV, s);
    for (int i = 0; i < NV; i++) snorm += s[i] * s[i];
    snorm = sqrt(snorm);
    /* the line: Gauss quadratic and each contact's cone terms */
    double Ms[NV], Js[BBO_MAXCON * 3], sMs = 0, sMdq = 0;
    for (int i = 0; i < NV; i++) { double t = 0; for (int j = 0; j < NV; j++) t += Mm[i * NV + j] * s[j]; Ms[i] = t; }
    for (int i = 0; i < NV; i++) { sMs += s[i] * Ms[i]; sMdq += s[i] * S.Mdq[i]; }
    for (int r = 0; r < nr; r++) { double t = 0; for (int d = 0; d < NV; d++) t += e->J[r][d] * s[d]; Js[r] = t; }
    for (int c = 0; c < e->nc; c++)
      cone_line_prep(&cl[c], S.jar + 3 * c, Js + 3 * c, e->mu[c], e->fr[c][0], e->fr[c][1], e->D + 3 * c);
    PrimalLine L;
    L.nc = e->nc; L.cl = cl;
    L.q0 = S.cost - total_cost(e, S.jar, S.force, NULL);  /* the Gauss part of the cost */
    L.q1 = sMdq; L.q2 = 0.5 * sMs;
    const double alpha = primal_search(&L, snorm, scale);
    if (g_flags & 256) fprintf(stderr, "   alpha %.6e evals %d\n", alpha, L.evals);
    if (alpha == 0) break;  /* no improvement */
    for (int i = 0; i < NV; i++) a[i] += alpha * s[i];
    const double oldcost = S.cost;
    primal_update(e, Mm, a0, a, &S);
    double gn = 0;
    for (int i = 0; i < NV; i++) gn += S.grad[i] * S.grad[i];
    if (scale * (oldcost - S.cost) < g_tol || scale * sqrt(gn) < g_tol) { it++; break; }
  }
  return it;
}

/* mj_fwdConstraint's warm start for the primal solvers: qacc_warmstart if its
 * total cost (Gauss + constraint) is not above the constraint cost of qacc_smooth
 * (whose Gauss cost is 0), else qacc_smooth [MJ] */
static void warmstart_choice(const Efc* e, const double* Mm, const double* a0, const double* warm, double* a) {
  static __thread PrimalState S;
  primal_update(e, Mm, a0, warm, &S);
  const double cw = S.cost;
  primal_update(e, Mm, a0, a0, &S);
  memcpy(a, cw > S.cost ? a0 : warm, NV * sizeof(double));
}

/* -------------------------------------------------------------- forward */
typedef struct {
  double xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], xI[NB][9];
  double xanchor[3][3], xaxis[3][3];
  double scom[NB][3], cinert[NB][36], cdof[NV][6], cdof_dot[NV][6], cvel[NB][6];
  double M[NV * NV];
} Work;

static void forward_impl(const double* qpos, const double* qvel, const double* ctrl, double* warm_io,
                         const float* hf, double size_z, bbo_forward_out* out) {
  compile_model();
  Model* m = &M_;
  static __thread Work W_;
  Work* w = &W_;
  BBO_PHASE(0);
  kinematics_all(qpos, w->xpos, w->xquat, w->xmat, w->xipos, w->xI, w->xanchor, w->xaxis);
  build_M(w->xmat, w->xpos, w->xipos, w->xI, w->xanchor, w->xaxis, w->scom, w->cinert, w->cdof, w->M);

  /* mj_comVel: cvel, cdof_dot */
  memset(w->cvel, 0, sizeof w->cvel);
  for (int b = 1; b < NB; b++) {
    int p = body_parent[b];
    double cv[6];
    memcpy(cv, w->cvel[p], sizeof cv);
    if (b == 1 || b == 7) {
      int da = (b == 1) ? 0 : 9;
      for (int i = 0; i < 3; i++) { memset(w->cdof_dot[da + i], 0, 6 * sizeof(double)); }
      for (int i = 0; i < 3; i++) for (int j = 0; j < 6; j++) cv[j] += w->cdof[da + i][j] * qvel[da + i];
      for (int i = 3; i < 6; i++) cross_motion(w->cdof_dot[da + i], cv, w->cdof[da + i]);
      for (int i = 3; i < 6; i++) for (int j = 0; j < 6; j++) cv[j] += w->cdof[da + i][j] * qvel[da + i];
    } else if (b >= 4) {
      int d = 6 + (b - 4);
      cross_motion(w->cdof_dot[d], cv, w->cdof[d]);
      for (int j = 0; j < 6; j++) cv[j] += w->cdof[d][j] * qvel[d];
    }
    memcpy(w->cvel[b], cv, sizeof cv);
  }

  /* mj_rne(flg_acc = 0): qfrc_bias */
  double cacc[NB][6], cfrc[NB][6];
  memset(cacc, 0, sizeof cacc);
  if (!(g_flags & BBO_DISABLE_GRAVITY)) cacc[0][5] = GRAVITY;
  for (int b = 1; b < NB; b++) {
    int p = body_parent[b];
    memcpy(cacc[b], cacc[p], 6 * sizeof(double));
    for (int d = 0; d < NV; d++)
      if (dof_body(d) == b)
        for (int j = 0; j < 6; j++) cacc[b][j] += w->cdof_dot[d][j] * qvel[d];
    double Iv[6], t1[6], t2[6];
    mul6(t1, w->cinert[b], cacc[b]);
    mul6(Iv, w->cinert[b], w->cvel[b]);
    cross_force(t2, w->cvel[b], Iv);
    for (int j = 0; j < 6; j++) cfrc[b][j] = t1[j] + t2[j];
  }
  for (int b = NB - 1; b >= 1; b--) {
    int p = body_parent[b];
    if (p > 0) for (int j = 0; j < 6; j++) cfrc[p][j] += cfrc[b][j];
  }
  double bias[NV], fsmooth[NV], a0[NV];
  for (int d = 0; d < NV; d++) {
    int b = dof_body(d);
    double s = 0;
    for (int j = 0; j < 6; j++) s += w->cdof[d][j] * cfrc[b][j];
    bias[d] = s;
  }
  for (int d = 0; d < NV; d++) fsmooth[d] = -bias[d];
  for (int k = 0; k < 3; k++) {
    if (!(g_flags & BBO_DISABLE_DAMPING)) fsmooth[6 + k] -= HINGE_DAMPING * qvel[6 + k];
    fsmooth[6 + k] += ctrl ? ctrl[k] : 0;
  }
  double L[NV * NV];
  memcpy(L, w->M, sizeof L);
  chol(L, NV);
  memcpy(a0, fsmooth, sizeof a0);
  chol_solve(L, NV, a0);

  /* collision + constraints */
  Contact con[BBO_MAXCON];
  int nground = 0, nbody = 0, overflow = 0;
  int nc = 0;
  BBO_PHASE(1);
  if (!(g_flags & BBO_DISABLE_CONTACT)) nc = collide(w->xpos, w->xmat, hf, size_z, con, &nground, &nbody, &overflow);
  BBO_PHASE(2);
  static __thread Efc E;
  E.nc = nc;
  const double dmax = 0.95, tc = fmax(0.02, 2 * TIMESTEP), dr = 1.0;
  const double K = 1 / fmax(MJMINVAL, dmax * dmax * tc * tc * dr * dr), Bd = 2 / fmax(MJMINVAL, dmax * tc);
  for (int c = 0; c < nc; c++) {
    Contact* cc = &con[c];
    /* jacdif = jac(body2, pos) - jac(body1, pos); body1 = ball for wheel pairs, world for hfield */
    double jd[3][NV];
    memset(jd, 0, sizeof jd);
    int b2 = cc->body2, b1 = cc->body1;
    for (int side = 0; side < 2; side++) {
      int b = side == 0 ? b2 : b1;
      double sg = side == 0 ? 1 : -1;
      if (b == 0) continue;
      for (int d = 0; d < NV; d++) {
        if (!dof_in_chain(d, b)) continue;
        double off[3], x[3];
        v3sub(off, cc->pos, w->scom[body_root[b]]);
        v3cross(x, w->cdof[d], off);
        for (int i = 0; i < 3; i++) jd[i][d] += sg * (w->cdof[d][3 + i] + x[i]);
      }
    }
    for (int rr = 0; rr < 3; rr++)
      for (int d = 0; d < NV; d++) E.J[3 * c + rr][d] = cc->frame[3 * rr] * jd[0][d] + cc->frame[3 * rr + 1] * jd[1][d] + cc->frame[3 * rr + 2] * jd[2][d];
    double tran = m->invweight_tran[b1] + m->invweight_tran[b2];
    double imp = impedance(cc->dist);
    if (imp < MJMINIMP) imp = MJMINIMP;
    if (imp > MJMAXIMP) imp = MJMAXIMP;
    double R0 = fmax(MJMINVAL, (1 - imp) * tran / imp);
    double R1 = R0 / 1.0; /* impratio = 1 */
    double mu = cc->fr[0] * sqrt(R1 / R0);
    double R2 = R1 * cc->fr[0] * cc->fr[0] / (cc->fr[1] * cc->fr[1]);
    E.D[3 * c] = 1 / R0; E.D[3 * c + 1] = 1 / R1; E.D[3 * c + 2] = 1 / R2;
    E.mu[c] = mu; E.fr[c][0] = cc->fr[0]; E.fr[c][1] = cc->fr[1];
    for (int rr = 0; rr < 3; rr++) {
      double vel = 0;
      for (int d = 0; d < NV; d++) vel += E.J[3 * c + rr][d] * qvel[d];
      double pos = rr == 0 ? cc->dist : 0;
      E.aref[3 * c + rr] = -Bd * vel - K * imp * pos;
    }
  }
  double a[NV];
  int niter = 0;
  if (nc == 0) memcpy(a, a0, sizeof a);
  else {
    int finite = warm_io != NULL;
    for (int i = 0; finite && i < NV; i++) finite = isfinite(warm_io[i]);
    if (finite && !(g_flags & BBO_WARM_ONLY)) warmstart_choice(&E, w->M, a0, warm_io, a);
    else if (finite) memcpy(a, warm_io, sizeof a);  /* the kernel's start: always the warm start */
    else memcpy(a, a0, sizeof a);
    BBO_PHASE(3);
    niter = newton(&E, w->M, a0, a, 1.0 / (m->meaninertia * NV));
  }
  BBO_PHASE(4);
  if (warm_io) memcpy(warm_io, a, sizeof a);

  if (out) {
    memcpy(out->qacc, a, sizeof a);
    memcpy(out->qacc_smooth, a0, sizeof a0);
    memcpy(out->qfrc_bias, bias, sizeof bias);
    memcpy(out->M, w->M, sizeof w->M);
    v3copy(out->xpos_base, w->xpos[1]);
    memcpy(out->xquat_base, w->xquat[1], 4 * sizeof(double));
    memcpy(out->cvel_base, w->cvel[1], 6 * sizeof(double));
    v3copy(out->subtree_com_base, w->scom[1]);
    out->ncon = nc; out->nground = nground; out->niter = niter; out->ground_overflow = overflow;
    out->nbody = nbody;
    for (int c = 0; c < nc && c < BBO_MAXCON; c++) {
      out->con_dist[c] = con[c].dist;
      memcpy(out->con_pos + 3 * c, con[c].pos, 3 * sizeof(double));
      memcpy(out->con_frame + 9 * c, con[c].frame, 9 * sizeof(double));
      out->con_body2[c] = con[c].body2;
      out->con_body1[c] = con[c].body1;
    }
    /* efc_force of each contact (contact frame: normal, then the two tangents) at the solution */
    {
      static __thread double jar[BBO_MAXCON * 3], frc[BBO_MAXCON * 3];
      for (int r = 0; r < 3 * nc; r++) { double s = -E.aref[r]; for (int d = 0; d < NV; d++) s += E.J[r][d] * a[d]; jar[r] = s; }
      total_cost(&E, jar, frc, NULL);
      memcpy(out->con_force, frc, 3 * nc * sizeof(double));
    }
    double ek = 0;
    for (int i = 0; i < NV; i++) for (int j = 0; j < NV; j++) ek += 0.5 * qvel[i] * w->M[i * NV + j] * qvel[j];
    double ep = 0;
    for (int b = 1; b < NB; b++) ep += m->mass[b] * GRAVITY * w->xipos[b][2];
    out->energy_kin = ek; out->energy_pot = ep;
  }
}

void bbo_forward(const double* qpos, const double* qvel, const double* ctrl, const double* warm,
                 const float* hfield, double size_z, bbo_forward_out* out) {
  double w[NV];
  if (warm) memcpy(w, warm, sizeof w);
  forward_impl(qpos, qvel, ctrl, warm ? w : NULL, hfield, size_z, out);
}

/* Momentum of the bodies (invariant tests): per tree the spatial
 * momentum sum_b cinert_b cvel_b about the tree's subtree COM (cvel_b = sum of the
 * chain's cdof qvel), moved to the system COM.  Hinge armature is joint-space
 * inertia invariant under a rigid motion of the whole, so these bodies' momenta are
 * what gravity-free, contact-free, undamped motion conserves. */
void bbo_momentum(const double* qpos, const double* qvel, double* out) {
  compile_model();
  Model* m = &M_;
  static __thread Work W_;
  Work* w = &W_;
  kinematics_all(qpos, w->xpos, w->xquat, w->xmat, w->xipos, w->xI, w->xanchor, w->xaxis);
  build_M(w->xmat, w->xpos, w->xipos, w->xI, w->xanchor, w->xaxis, w->scom, w->cinert, w->cdof, w->M);
  double h[2][6] = {{0}}, mt = 0, c[3] = {0, 0, 0};
  for (int b = 1; b < NB; b++) {
    double cv[6] = {0, 0, 0, 0, 0, 0};
    for (int d = 0; d < NV; d++)
      if (dof_in_chain(d, b)) for (int j = 0; j < 6; j++) cv[j] += w->cdof[d][j] * qvel[d];
    const int t = b == 7;
    for (int i = 0; i < 6; i++) { double s = 0; for (int j = 0; j < 6; j++) s += w->cinert[b][6 * i + j] * cv[j]; h[t][i] += s; }
    mt += m->mass[b];
    for (int i = 0; i < 3; i++) c[i] += m->mass[b] * w->xipos[b][i];
  }
  for (int i = 0; i < 3; i++) c[i] /= mt;
  double L[3] = {0, 0, 0}, P[3] = {0, 0, 0};
  for (int t = 0; t < 2; t++) {
    double r[3], x[3];
    v3sub(r, w->scom[t == 0 ? 1 : 7], c);
    v3cross(x, r, h[t] + 3);
    for (int i = 0; i < 3; i++) { L[i] += h[t][i] + x[i]; P[i] += h[t][3 + i]; }
  }
  v3copy(out, P); v3copy(out + 3, L); v3copy(out + 6, c);
}

/* mj_integratePos */
static void integrate_pos(double* qpos, const double* v, double h) {
  for (int t = 0; t < 2; t++) {
    int qa = t == 0 ? 0 : 10, da = t == 0 ? 0 : 9;
    for (int i = 0; i < 3; i++) qpos[qa + i] += h * v[da + i];
    quat_integrate(qpos + qa + 3, v + da + 3, h);
  }
  for (int k = 0; k < 3; k++) qpos[7 + k] += h * v[6 + k];
}

/* MuJoCo's mju_isBad over x[0..n): NaN or |x| > mjMAXVAL (1e10) */
static int vec_bad(const double* x, int n) {
  for (int i = 0; i < n; i++) if (!(fabs(x[i]) <= 1e10)) return 1;
  return 0;
}

/* mj_resetData for this model: qpos0, zero qvel, qacc_warmstart and ctrl (no
 * reset height offset: that is the env's, ballbot_env.py:616-617) */
static void reset_data(double* qpos, double* qvel, double* warm, double* ctrl) {
  compile_model();
  memcpy(qpos, M_.qpos0, NQ * sizeof(double));
  memset(qvel, 0, NV * sizeof(double));
  if (warm) memset(warm, 0, NV * sizeof(double));
  ctrl[0] = ctrl[1] = ctrl[2] = 0;
}

/* BBO_RKMK: replace the free joints' body angular velocities in x (dofs 3..6, 12..15)
 * by dexp^-1_{-theta}(w) for the stage's rotation vectors theta[0..3) (base), [3..6) (ball) */
static void rkmk_rates(double* x, const double* theta) {
  for (int t = 0; t < 2; t++) {
    double* w = x + (t ? 9 : 0) + 3;
    const double* th = theta + 3 * t;
    double c1[3], c2[3];
    v3cross(c1, th, w);
    v3cross(c2, th, c1);
    for (int i = 0; i < 3; i++) w[i] += 0.5 * c1[i] + c2[i] / 12.0;
  }
}

/* mj_step with integrator RK4: mj_checkPos, mj_checkVel, mj_forward,
 * mj_checkAcc, then mj_RungeKutta(m, d, 4).  A bad qpos/qvel (before the
 * forward) or qacc (after it) resets the data (mj_resetData; the qacc case
 * then runs mj_forward again) and the step goes on from qpos0.  A bad ctrl
 * zeroes every ctrl (mjWARN_BADCTRL, mj_fwdActuation).  Returns 1 if a
 * divergence reset happened. */
int bbo_mj_step(double* qpos, double* qvel, double* warm, const double* ctrl_in,
                const float* hfield, double size_z, bbo_forward_out* stage4) {
  static const double A[3] = {0.5, 0.5, 1.0}; /* RK4 A (sub)diagonal */
  static const double B[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6};
  const double h = TIMESTEP;
  double q0[NQ], v0[NV], X[4][NV], F[4][NV], ctrl[3] = {ctrl_in[0], ctrl_in[1], ctrl_in[2]};
  int reset = 0;
  if (vec_bad(ctrl, 3)) ctrl[0] = ctrl[1] = ctrl[2] = 0;
  if (vec_bad(qpos, NQ) || vec_bad(qvel, NV)) { reset_data(qpos, qvel, warm, ctrl); reset = 1; }
  memcpy(q0, qpos, sizeof q0);
  memcpy(v0, qvel, sizeof v0);
  bbo_forward_out tmp;
  bbo_forward_out* o = stage4 ? stage4 : &tmp;
  forward_impl(q0, v0, ctrl, warm, hfield, size_z, o);
  if (!reset && vec_bad(o->qacc, NV)) {
    reset_data(q0, v0, warm, ctrl);
    reset = 1;
    forward_impl(q0, v0, ctrl, warm, hfield, size_z, o);
  }
  memcpy(X[0], v0, sizeof v0);
  memcpy(F[0], o->qacc, sizeof F[0]);
  /* BBO_RKMK (test-only): the free joints' rotation rates of stage j become
   * dexp^-1_{-theta_j}(w_j) = w + theta x w / 2 + theta x (theta x w) / 12, theta_j
   * the stage's rotation vector from the step's start orientation (q_j = q0 exp(theta_j)) */
  const int rkmk = (g_flags & BBO_RKMK) != 0;
  double th[4][6];
  memset(th, 0, sizeof th);
  if (rkmk) rkmk_rates(X[0], th[0]);
  for (int i = 1; i < 4; i++) {
    double dxv[NV], dxa[NV], q[NQ], v[NV];
    for (int d = 0; d < NV; d++) { dxv[d] = A[i - 1] * X[i - 1][d]; dxa[d] = A[i - 1] * F[i - 1][d]; }
    if (rkmk)
      for (int t = 0; t < 2; t++)
        for (int c = 0; c < 3; c++) {
          th[i][3 * t + c] = h * dxv[(t ? 9 : 0) + 3 + c];
        }
    memcpy(q, q0, sizeof q);
    integrate_pos(q, dxv, h);
    for (int d = 0; d < NV; d++) v[d] = v0[d] + h * dxa[d];
    forward_impl(q, v, ctrl, warm, hfield, size_z, o);
    memcpy(X[i], v, sizeof v);
    memcpy(F[i], o->qacc, sizeof F[i]);
    if (rkmk) rkmk_rates(X[i], th[i]);
  }
  double dv[NV], da[NV];
  for (int d = 0; d < NV; d++) {
    dv[d] = B[0] * X[0][d] + B[1] * X[1][d] + B[2] * X[2][d] + B[3] * X[3][d];
    da[d] = B[0] * F[0][d] + B[1] * F[1][d] + B[2] * F[2][d] + B[3] * F[3][d];
  }
  /* mj_advance: qvel += h*qacc_rk, integratePos(qpos, v_rk, h) */
  for (int d = 0; d < NV; d++) qvel[d] = v0[d] + h * da[d];
  memcpy(qpos, q0, sizeof q0);
  integrate_pos(qpos, dv, h);
  return reset;
}

/* ---------------------------------------------------------------- env glue */
void bbo_quat_to_rotvec(const double* q, double* rv) {
  /* numpy-quaternion: as_rotation_vector(q) = 2 * log(q).vec ; quaternion_log */
  const double EPS = 1e-14;
  double b = sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (fabs(b) <= EPS * fabs(q[0])) {
    if (q[0] < 0) { rv[0] = 2 * PI; rv[1] = rv[2] = 0; }
    else { rv[0] = rv[1] = rv[2] = 0; }
    return;
  }
  double v = atan2(b, q[0]), f = v / b;
  rv[0] = 2 * f * q[1]; rv[1] = 2 * f * q[2]; rv[2] = 2 * f * q[3];
}

static float clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

void bbo_reset_state(double offset, double* qpos, double* qvel, double* warm) {
  compile_model();
  memcpy(qpos, M_.qpos0, NQ * sizeof(double));
  qpos[2] += offset;   /* ballbot_env.py:616 */
  qpos[12] += offset;  /* ballbot_env.py:617 */
  memset(qvel, 0, NV * sizeof(double));
  if (warm) memset(warm, 0, NV * sizeof(double));
}

double bbo_init_offset(const float* hf, double size_z) {
  /* ballbot_env.py:527-565 with the ball geom at (0,0,0.12) after mj_forward(qpos0) */
  const int n = BBO_HF_N;
  double sz = HF_SIZE[0];
  double cell = sz / n;          /* quirk: size/nrows, not 2*size/(nrows-1) */
  int center = n / 2;
  double amin[2] = {-BALL_R, -BALL_R}, amax[2] = {BALL_R, BALL_R};
  int x0 = center - abs((int)floor(amin[0] / cell));
  int x1 = center + (int)floor(amax[0] / cell) + 1;
  int y0 = center - abs((int)floor(amin[1] / cell));
  int y1 = center + (int)floor(amax[1] / cell) + 1;
  double mx = -1e300;
  for (int i = x0; i < x1; i++)
    for (int j = y0; j < y1; j++) { double v = hf ? (double)hf[i * n + j] : 0.0; if (v > mx) mx = v; }
  return mx * size_z + 0.01;
}

int bbo_env_step(const bbo_env_cfg* cfg, double* qpos, double* qvel, double* warm, int* step_counter,
                 const float* action, const float* hfield, double size_z, float* obs15, float* reward,
                 float* pos2d, double* tilt_deg) {
  /* action -> ctrl (ballbot_env.py:903-907): f32 math, then negated into f64 ctrl */
  float mwv = (float)cfg->max_wheel_velocity;
  double ctrl[3];
  for (int k = 0; k < 3; k++) {
    float c = action[k] * mwv;
    c = clipf(c, -mwv, mwv);
    ctrl[k] = -(double)c;
  }
  bbo_forward_out s4;
  /* mj_step's divergence reset (mj_checkPos/Vel/Acc) happens inside it; the
   * episode goes on from qpos0 with step_counter unchanged: mj_step advances
   * time past 0, so the env's time==0 check (ballbot_env.py:897-899) stays off */
  int diverged = bbo_mj_step(qpos, qvel, warm, ctrl, hfield, size_z, &s4);

  /* _get_obs (ballbot_env.py:771-811) from stage-4 xquat/cvel and final qvel */
  double rv[3];
  bbo_quat_to_rotvec(s4.xquat_base, rv);
  float orient[3] = {(float)rv[0], (float)rv[1], (float)rv[2]};
  float motor[3];
  for (int k = 0; k < 3; k++) { /* qvel[joint id k+1]: base dofs 1,2,3 */
    float v = (float)qvel[1 + k];
    v = v / mwv;
    motor[k] = clipf(v, -2.0f, 2.0f);
  }
  float vel[3], angv[3];
  for (int i = 0; i < 3; i++) {
    vel[i] = clipf((float)s4.cvel_base[i], -2.0f, 2.0f);
    angv[i] = clipf((float)s4.cvel_base[3 + i], -2.0f, 2.0f);
  }
  /* sorted keys: actions, angular_vel, motor_state, orientation, vel */
  for (int i = 0; i < 3; i++) {
    obs15[i] = action[i]; obs15[3 + i] = angv[i]; obs15[6 + i] = motor[i];
    obs15[9 + i] = orient[i]; obs15[12 + i] = vel[i];
  }
  if (pos2d) { pos2d[0] = (float)s4.xpos_base[0]; pos2d[1] = (float)s4.xpos_base[1]; }

  /* reward (ballbot_env.py:929-937 + DirectionalReward) in float32 */
  float dir = vel[0] * cfg->target_dir[0] + vel[1] * cfg->target_dir[1];
  float r = dir * cfg->reward_scale;
  float nrm = sqrtf(action[0] * action[0] + action[1] * action[1] + action[2] * action[2]);
  float reg = cfg->action_reg_coef * (nrm * nrm);
  r = r + reg;
  *step_counter += 1;
  int terminated = (*step_counter >= cfg->max_ep_steps);
  /* tilt (ballbot_env.py:989-1008): R from f32 rotvec (f64 math) -> arccos(R22) */
  double rx = orient[0], ry = orient[1], rz = orient[2];
  double th = sqrt(rx * rx + ry * ry + rz * rz) / 2;
  double qw = cos(th), sf = th > 0 ? sin(th) / th : 1.0;
  double qx = sf * rx / 2, qy = sf * ry / 2, qz = sf * rz / 2;
  double nn = qw * qw + qx * qx + qy * qy + qz * qz;
  double R22 = 1 - 2 * (qx * qx + qy * qy) / nn;
  double ang = acos(R22) * 180 / PI;
  if (tilt_deg) *tilt_deg = ang;
  int failure = ang > cfg->max_allowed_tilt;
  if (failure) terminated = 1;
  else r = r + cfg->survival_bonus;
  *reward = r;
  return (terminated ? 1 : 0) | (failure ? 2 : 0) | (diverged ? 4 : 0);
}

int bbo_env_step_batch(const bbo_env_cfg* cfg, int n, double* qpos, double* qvel, double* warm,
                       int* step_counter, const float* actions, const float* hfield, double size_z,
                       float* obs, float* reward, unsigned char* done, double offset) {
  int nd = 0;
  for (int e = 0; e < n; e++) {
    double* q = qpos + e * NQ; double* v = qvel + e * NV; double* w = warm + e * NV;
    int f = bbo_env_step(cfg, q, v, w, step_counter + e, actions + 3 * e, hfield, size_z, obs + 15 * e,
                         reward + e, NULL, NULL);
    done[e] = (unsigned char)(f & 7);
    if (f & 1) { /* terminated -> auto-reset (a divergence reset ends nothing) */
      bbo_reset_state(offset, q, v, w);
      step_counter[e] = 0;
      nd++;
    }
  }
  return nd;
}

/* the same, one env per OpenMP thread (independent envs; the CPU baseline on
 * all granted host cores) */
int bbo_env_step_batch_mt(const bbo_env_cfg* cfg, int n, double* qpos, double* qvel, double* warm,
                          int* step_counter, const float* actions, const float* hfield, double size_z,
                          float* obs, float* reward, unsigned char* done, double offset, int threads) {
  compile_model(); /* once, before the threads share the model */
  int nd = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 4) reduction(+ : nd)
  for (int e = 0; e < n; e++) {
    double* q = qpos + e * NQ; double* v = qvel + e * NV; double* w = warm + e * NV;
    int f = bbo_env_step(cfg, q, v, w, step_counter + e, actions + 3 * e, hfield, size_z, obs + 15 * e,
                         reward + e, NULL, NULL);
    done[e] = (unsigned char)(f & 7);
    if (f & 1) {
      bbo_reset_state(offset, q, v, w);
      step_counter[e] = 0;
      nd++;
    }
  }
  return nd;
}

/* ------------------------------------------------------------ depth cameras
 * Restates what RGBDInputs (sensors/rgbd.py:46-82) reads from MuJoCo's
 * renderer for cam_0 / cam_1 (ballbot.xml:44-54): the linear eye-space depth
 * (z along the camera's -z axis, mujoco.Renderer's near/(1 - z(1 - near/far))
 * conversion of the depth buffer), one sample per pixel centre, fovy 90,
 * clipped to <= 1.0 (rgbd.py:74).  Visible geoms (groups 0-2): the hfield,
 * the ball, the tower cylinder, the cam sticks and the wheel capsules; the
 * ballast (group 3) is hidden and the cone meshes are missing from the
 * reference.  Back faces are culled (a ray starting inside a geom does not see
 * it), surfaces nearer than znear = 1e-4 * extent (extent 10*sqrt(2), the
 * model's comment at ballbot.xml:9) are clipped.  The hfield surface is
 * triangulated as the collision prisms (cell (r,c): (r,c)(r+1,c)(r,c+1) and
 * (r+1,c)(r,c+1)(r+1,c+1)); its side walls are not drawn.  Row 0 = top of the
 * image (x right, y up in the camera frame).  PARITY UNPINNED against
 * MuJoCo's OpenGL rasteriser (not available); tests pin it by analytic scenes.
 */
#define BBO_ZNEAR (1e-4 * 14.142135623730951)

static double ray_sphere(const double* o, const double* d, const double* c, double r) {
  double oc[3]; v3sub(oc, o, c);
  double b = v3dot(oc, d), cc = v3dot(oc, oc) - r * r, h = b * b - cc;
  if (h < 0) return -1;
  return -b - sqrt(h);
}

/* front-face entry of a capsule (segment pa-pb, radius r); -1 if none; |d| = 1 */
static double ray_capsule(const double* o, const double* d, const double* pa, const double* pb, double r) {
  double ba[3], oa[3];
  v3sub(ba, pb, pa); v3sub(oa, o, pa);
  double baba = v3dot(ba, ba), bard = v3dot(ba, d), baoa = v3dot(ba, oa), rdoa = v3dot(d, oa), oaoa = v3dot(oa, oa);
  double a = baba - bard * bard, b = baba * rdoa - baoa * bard, c = baba * oaoa - baoa * baoa - r * r * baba;
  double h = b * b - a * c;
  if (h < 0) return -1;
  double t = a > 1e-300 ? (-b - sqrt(h)) / a : -1;
  double y = baoa + t * bard;
  if (a > 1e-300 && y > 0 && y < baba) return t;
  /* caps: the sphere at the end the body hit falls beyond */
  double oc[3];
  if (y <= 0) v3copy(oc, oa); else v3sub(oc, o, pb);
  double bb = v3dot(d, oc), cc = v3dot(oc, oc) - r * r, hh = bb * bb - cc;
  if (hh > 0) return -bb - sqrt(hh);
  return -1;
}

/* front-face entry of a capped cylinder (axis pa-pb, radius r); -1 if none; |d| = 1 */
static double ray_cylinder(const double* o, const double* d, const double* pa, const double* pb, double r) {
  double ba[3], oc[3];
  v3sub(ba, pb, pa); v3sub(oc, o, pa);
  double baba = v3dot(ba, ba), bard = v3dot(ba, d), baoc = v3dot(ba, oc);
  double k2 = baba - bard * bard, k1 = baba * v3dot(oc, d) - baoc * bard;
  double k0 = baba * v3dot(oc, oc) - baoc * baoc - r * r * baba;
  double h = k1 * k1 - k2 * k0;
  if (h < 0) return -1;
  h = sqrt(h);
  if (k2 > 1e-300) {
    double t = (-k1 - h) / k2, y = baoc + t * bard;
    if (y > 0 && y < baba) return t;
    if (fabs(bard) < 1e-300) return -1;
    t = (((y < 0) ? 0 : baba) - baoc) / bard;
    if (fabs(k1 + k2 * t) < h) return t;
    return -1;
  }
  /* ray parallel to the axis: caps only */
  if (k0 > 0 || fabs(bard) < 1e-300) return -1;
  double t0 = (0 - baoc) / bard, t1 = (baba - baoc) / bard;
  return t0 < t1 ? t0 : t1;
}

/* two-sided Moller-Trumbore; -1 if none */
static double ray_tri(const double* o, const double* d, const double* a, const double* b, const double* c) {
  double e1[3], e2[3], p[3], s[3], q[3];
  v3sub(e1, b, a); v3sub(e2, c, a);
  v3cross(p, d, e2);
  double det = v3dot(e1, p);
  if (fabs(det) < 1e-300) return -1;
  double inv = 1.0 / det;
  v3sub(s, o, a);
  double u = v3dot(s, p) * inv;
  if (u < 0 || u > 1) return -1;
  v3cross(q, s, e1);
  double v = v3dot(d, q) * inv;
  if (v < 0 || u + v > 1) return -1;
  return v3dot(e2, q) * inv;
}

static double hf_z(const float* hf, int r, int c, double size_z) { return (double)hf[r * BBO_HF_N + c] * size_z; }

/* nearest hfield hit along o + t d (|d| = 1) for t in (tmin, tmax); -1 if none.
 * 2-D DDA over the cells the ray's xy projection crosses. */
static double ray_hfield(const double* o, const double* d, const float* hf, double size_z, double tmin, double tmax) {
  const int N1 = BBO_HF_N - 1;
  const double sx = HF_SIZE[0], sy = HF_SIZE[1], dx = 2 * sx / N1, dy = 2 * sy / N1;
  /* clip the parameter range to the field's xy box */
  double t0 = tmin, t1 = tmax;
  for (int ax = 0; ax < 2; ax++) {
    double lo = -HF_SIZE[ax], hi = HF_SIZE[ax];
    if (fabs(d[ax]) < 1e-300) { if (o[ax] < lo || o[ax] > hi) return -1; continue; }
    double ta = (lo - o[ax]) / d[ax], tb = (hi - o[ax]) / d[ax];
    if (ta > tb) { double s = ta; ta = tb; tb = s; }
    if (ta > t0) t0 = ta;
    if (tb < t1) t1 = tb;
  }
  if (t0 > t1) return -1;
  double px = o[0] + t0 * d[0], py = o[1] + t0 * d[1];
  int c = (int)floor((px + sx) / dx), r = (int)floor((py + sy) / dy);
  c = c < 0 ? 0 : (c > N1 - 1 ? N1 - 1 : c);
  r = r < 0 ? 0 : (r > N1 - 1 ? N1 - 1 : r);
  int stc = d[0] > 0 ? 1 : -1, str = d[1] > 0 ? 1 : -1;
  double tdx = fabs(d[0]) > 1e-300 ? dx / fabs(d[0]) : 1e300, tdy = fabs(d[1]) > 1e-300 ? dy / fabs(d[1]) : 1e300;
  double nx = -sx + (c + (stc > 0 ? 1 : 0)) * dx, ny = -sy + (r + (str > 0 ? 1 : 0)) * dy;
  double tmx = fabs(d[0]) > 1e-300 ? (nx - o[0]) / d[0] : 1e300, tmy = fabs(d[1]) > 1e-300 ? (ny - o[1]) / d[1] : 1e300;
  for (int it = 0; it < 4 * BBO_HF_N; it++) {
    double x0 = -sx + c * dx, x1 = -sx + (c + 1) * dx, y0 = -sy + r * dy, y1 = -sy + (r + 1) * dy;
    double A[3] = {x0, y0, hf_z(hf, r, c, size_z)}, B[3] = {x0, y1, hf_z(hf, r + 1, c, size_z)};
    double C[3] = {x1, y0, hf_z(hf, r, c + 1, size_z)}, D[3] = {x1, y1, hf_z(hf, r + 1, c + 1, size_z)};
    double best = -1;
    double ta = ray_tri(o, d, A, B, C), tb = ray_tri(o, d, B, C, D);
    if (ta > tmin && ta < tmax) best = ta;
    if (tb > tmin && tb < tmax && (best < 0 || tb < best)) best = tb;
    if (best > 0) return best;
    double tn = tmx < tmy ? tmx : tmy;
    if (tn > t1) break;
    if (tmx < tmy) { c += stc; tmx += tdx; if (c < 0 || c > N1 - 1) break; }
    else { r += str; tmy += tdy; if (r < 0 || r > N1 - 1) break; }
  }
  return -1;
}

/* camera frames in their bodies (ballbot.xml:47,53: pos 0, euler 180 0 0) */
void bbo_render_depth(const double* qpos, const float* hf, double size_z, int cam, int H, int W, float* out) {
  double xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], xI[NB][9], xanchor[3][3], xaxis[3][3];
  kinematics_all(qpos, xpos, xquat, xmat, xipos, xI, xanchor, xaxis);
  int b = 2 + cam;
  double qc[4], cq[4], R[9];
  euler2quat(qc, 180, 0, 0);
  qmul(cq, xquat[b], qc);
  q2mat(R, cq);
  const double* o = xpos[b];
  Convex g[6]; int cyl[6], body[6];
  body_geoms(xpos, xmat, g, cyl, body);
  double ball[3], t[3];
  m3v(t, xmat[7], BALL_GPOS);
  v3add(ball, xpos[7], t);
  const double tanh_ = 1.0; /* tan(fovy / 2), fovy 90 */
  for (int i = 0; i < H; i++)
    for (int j = 0; j < W; j++) {
      double xc = (2.0 * (j + 0.5) / W - 1.0) * tanh_ * ((double)W / H);
      double yc = (1.0 - 2.0 * (i + 0.5) / H) * tanh_;
      double dc[3] = {xc, yc, -1.0}, d[3];
      m3v(d, R, dc);
      double len = sqrt(v3dot(d, d));
      for (int k = 0; k < 3; k++) d[k] /= len;
      const double tmin = BBO_ZNEAR * len, tmax = 1.0 * len;  /* z-depth in (znear, 1] */
      double best = tmax;
      double th = ray_sphere(o, d, ball, BALL_R);
      if (th > tmin && th < best) best = th;
      for (int k = 0; k < 6; k++) {
        double pa[3], pb[3];
        for (int q = 0; q < 3; q++) { pa[q] = g[k].c[q] - g[k].a[q] * g[k].hh; pb[q] = g[k].c[q] + g[k].a[q] * g[k].hh; }
        double tk = cyl[k] ? ray_cylinder(o, d, pa, pb, g[k].r) : ray_capsule(o, d, pa, pb, g[k].r);
        if (tk > tmin && tk < best) best = tk;
      }
      double tg = ray_hfield(o, d, hf, size_z, tmin, best);
      if (tg > tmin && tg < best) best = tg;
      double z = best / len;
      out[i * W + j] = (float)(z >= 1.0 ? 1.0 : z);
    }
}
