// Test-only host build of the product's per-env templates (bb_step.h), used
// to debug the kernel math against the oracle on a machine without a GPU.
// Never shipped, never loaded by the product path.
#include <vector>
#include "bb_model.h"
#include "bb_step.h"

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

extern "C" {
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
}
