// flopcount.cpp -- algorithmic FLOP counter for the oracle's env step (test
// infrastructure, SURVEY.md §8 D3/D4: "Algorithmic FLOPs are counted by an
// op-counter in the CPU oracle per config and recorded next to the bytes").
//
// bb_oracle.c (the fp64 restatement of mj_step + env glue) is compiled a second
// time as C++ with `double` replaced by FD, a double that counts the arithmetic
// done on it: add/sub, mul, div, sqrt, transcendentals (sin, cos, tan, atan2,
// acos, exp, log, pow) and comparisons, separately.  The counted work is the
// oracle's own algorithm (MuJoCo's: dense 15x15 Newton with Cholesky and an
// exact line search), i.e. the reference's work per env-step, not what the HIP
// kernels execute.  FLOP = add + sub + mul + div + sqrt + transcendental (one
// each, the usual convention); comparisons are reported but not counted.
// Float32 glue arithmetic (reward, obs clipping) is not counted (a few dozen ops).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

namespace fc {
struct Counts {
  unsigned long long add, mul, div, sqrt, trans, cmp;
};
constexpr int NPH = 5;  // bb_oracle.c BBO_PHASE: kinematics/mass/bias, collision, assembly, solver, RK4/glue
// per thread: bbo_count_flops_replay runs on several host threads at once (tools/flops.py)
static thread_local Counts ph[NPH];
static thread_local Counts g;        // the phase being counted (copied back at every phase switch)
static thread_local int cur = 4;
inline void phase(int k) {
  Counts& a = ph[cur];
  a.add += g.add; a.mul += g.mul; a.div += g.div; a.sqrt += g.sqrt; a.trans += g.trans; a.cmp += g.cmp;
  g = Counts{};
  cur = k;
}
}  // namespace fc

struct FD {
  double v;
  FD() = default;
  constexpr FD(double x) : v(x) {}
  explicit operator double() const { return v; }
  explicit operator float() const { return float(v); }
  explicit operator int() const { return int(v); }
  explicit operator long() const { return long(v); }
  explicit operator unsigned() const { return unsigned(v); }
  FD& operator+=(FD o) { fc::g.add++; v += o.v; return *this; }
  FD& operator-=(FD o) { fc::g.add++; v -= o.v; return *this; }
  FD& operator*=(FD o) { fc::g.mul++; v *= o.v; return *this; }
  FD& operator/=(FD o) { fc::g.div++; v /= o.v; return *this; }
  FD operator-() const { return FD(-v); }
  FD operator+() const { return *this; }
};
static_assert(sizeof(FD) == sizeof(double), "FD must be layout-compatible with double");

#define FD_BIN(op, ctr)                                                              \
  inline FD operator op(FD a, FD b) { fc::g.ctr++; return FD(a.v op b.v); }         \
  inline FD operator op(FD a, double b) { fc::g.ctr++; return FD(a.v op b); }       \
  inline FD operator op(double a, FD b) { fc::g.ctr++; return FD(a op b.v); }       \
  inline FD operator op(FD a, int b) { fc::g.ctr++; return FD(a.v op b); }          \
  inline FD operator op(int a, FD b) { fc::g.ctr++; return FD(a op b.v); }          \
  inline FD operator op(FD a, float b) { fc::g.ctr++; return FD(a.v op b); }        \
  inline FD operator op(float a, FD b) { fc::g.ctr++; return FD(a op b.v); }
FD_BIN(+, add)
FD_BIN(-, add)
FD_BIN(*, mul)
FD_BIN(/, div)
#define FD_CMP(op)                                                                   \
  inline bool operator op(FD a, FD b) { fc::g.cmp++; return a.v op b.v; }            \
  inline bool operator op(FD a, double b) { fc::g.cmp++; return a.v op b; }          \
  inline bool operator op(double a, FD b) { fc::g.cmp++; return a op b.v; }          \
  inline bool operator op(FD a, int b) { fc::g.cmp++; return a.v op b; }             \
  inline bool operator op(int a, FD b) { fc::g.cmp++; return a op b.v; }             \
  inline bool operator op(FD a, float b) { fc::g.cmp++; return a.v op b; }           \
  inline bool operator op(float a, FD b) { fc::g.cmp++; return a op b.v; }
FD_CMP(<)
FD_CMP(>)
FD_CMP(<=)
FD_CMP(>=)
FD_CMP(==)
FD_CMP(!=)

inline FD sqrt(FD a) { fc::g.sqrt++; return FD(::sqrt(a.v)); }
inline FD fabs(FD a) { return FD(::fabs(a.v)); }
inline FD floor(FD a) { return FD(::floor(a.v)); }
inline FD ceil(FD a) { return FD(::ceil(a.v)); }
inline FD fmax(FD a, FD b) { fc::g.cmp++; return FD(::fmax(a.v, b.v)); }
inline FD fmin(FD a, FD b) { fc::g.cmp++; return FD(::fmin(a.v, b.v)); }
inline FD sin(FD a) { fc::g.trans++; return FD(::sin(a.v)); }
inline FD cos(FD a) { fc::g.trans++; return FD(::cos(a.v)); }
inline FD tan(FD a) { fc::g.trans++; return FD(::tan(a.v)); }
inline FD acos(FD a) { fc::g.trans++; return FD(::acos(a.v)); }
inline FD exp(FD a) { fc::g.trans++; return FD(::exp(a.v)); }
inline FD log(FD a) { fc::g.trans++; return FD(::log(a.v)); }
inline FD atan2(FD a, FD b) { fc::g.trans++; return FD(::atan2(a.v, b.v)); }
inline FD pow(FD a, FD b) { fc::g.trans++; return FD(::pow(a.v, b.v)); }
inline FD pow(FD a, double b) { fc::g.trans++; return FD(::pow(a.v, b)); }
inline FD pow(FD a, int b) { fc::g.trans++; return FD(::pow(a.v, b)); }
inline bool isfinite(FD a) { return ::isfinite(a.v); }
inline bool isnan(FD a) { return ::isnan(a.v); }

// the restatement, compiled over FD (its own headers were included above and
// are guarded; the debug prints are dropped)
#define fprintf(...) ((void)0)
#define BBO_PHASE(k) fc::phase(k)
#define double FD
#include "bb_oracle.c"
#undef double
#undef fprintf

extern "C" {

// Run n_burn uncounted then n_steps counted env-steps of n_envs envs (auto-reset
// on termination, as the product) from the reset state with actions uniform in [-scale, scale] (a fixed
// LCG, seed), on one heightfield, with MuJoCo's solver settings (tolerance 1e-8,
// line search to 0.01 within 50 evaluations; the oracle's parity runs solve to
// 1e-10 with a roundoff-exact line search).  out[30] = per env-step means of {add/sub,
// mul, div, sqrt, transcendental, comparisons} for each of the 5 phases
// (BBO_PHASE order); returns env-steps run.
long long bbo_count_flops(int n_envs, int n_burn, int n_steps, const float* hfield, double size_z, double offset,
                          double action_scale, unsigned seed, double* out) {
  compile_model();
  const int maxiter0 = g_maxiter, lsmax0 = g_lsmax;
  const FD tol0 = g_tol, lstol0 = g_lstol;
  g_maxiter = 100;  // MuJoCo defaults: iterations, tolerance, ls_iterations, ls_tolerance
  g_tol = 1e-8;
  g_lsmax = 50;
  g_lstol = 0.01;
  bbo_env_cfg cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.max_ep_steps = 4000;
  cfg.max_allowed_tilt = 20.0;
  cfg.max_wheel_velocity = 10.0;
  cfg.reward_scale = 0.01f;
  cfg.action_reg_coef = -0.0001f;
  cfg.survival_bonus = 0.02f;
  cfg.target_dir[0] = 0.0f;
  cfg.target_dir[1] = 1.0f;
  FD* q = (FD*)calloc((size_t)n_envs * NQ, sizeof(FD));
  FD* v = (FD*)calloc((size_t)n_envs * NV, sizeof(FD));
  FD* w = (FD*)calloc((size_t)n_envs * NV, sizeof(FD));
  int* sc = (int*)calloc((size_t)n_envs, sizeof(int));
  for (int e = 0; e < n_envs; e++) bbo_reset_state(FD(offset), q + e * NQ, v + e * NV, w + e * NV);
  uint64_t st = seed * 6364136223846793005ull + 1442695040888963407ull;
  long long steps = 0;
  for (int t = 0; t < n_burn + n_steps; t++)
    for (int e = 0; e < n_envs; e++) {
      if (t == n_burn && e == 0) {  // the steady-state mix of episode ages starts here
        fc::phase(4);
        fc::g = fc::Counts{};
        for (auto& c : fc::ph) c = fc::Counts{};
        fc::cur = 4;
        steps = 0;
      }
      float a[3], obs[15], r, p2[2];
      for (int k = 0; k < 3; k++) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        a[k] = (float)((((st >> 11) * (1.0 / 9007199254740992.0)) * 2 - 1) * action_scale);
      }
      int f = bbo_env_step(&cfg, q + e * NQ, v + e * NV, w + e * NV, sc + e, a, hfield, FD(size_z), obs, &r, p2,
                           nullptr);
      steps++;
      if (f & 1) {
        bbo_reset_state(FD(offset), q + e * NQ, v + e * NV, w + e * NV);
        sc[e] = 0;
      }
    }
  fc::phase(4);
  const double k = steps ? 1.0 / (double)steps : 0.0;
  for (int p = 0; p < fc::NPH; p++) {
    const fc::Counts& c = fc::ph[p];
    double* o = out + 6 * p;
    o[0] = c.add * k; o[1] = c.mul * k; o[2] = c.div * k; o[3] = c.sqrt * k; o[4] = c.trans * k; o[5] = c.cmp * k;
  }
  g_maxiter = maxiter0;
  g_tol = tol0;
  g_lsmax = lsmax0;
  g_lstol = lstol0;
  free(q); free(v); free(w); free(sc);
  return steps;
}

// Warm-up for threaded use: the model compiles once, outside the worker threads.
void bbo_count_prepare(void) {
  compile_model();
  g_maxiter = 100;  // MuJoCo defaults: iterations, tolerance, ls_iterations, ls_tolerance
  g_tol = 1e-8;
  g_lsmax = 50;
  g_lstol = 0.01;
}

// The bench's timed mix, replayed: n_envs envs from their states at the start of the timed window
// (q[n][17], v[n][15], w[n][15], step counters sc[n]; updated in place) step n_steps times with
// the window's own actions (actions[t][n][3]), auto-resetting onto the env's next terrain draw:
// env e starts on table[terr[e * max_ep]] and its k-th reset moves to table[terr[e * max_ep + k]]
// (the last one repeats past max_ep; *overrun counts such resets), each table slot a float32
// [293 * 293] heightfield with its init offset offsets[slot], vertical scale size_z.  Thread-safe
// (thread-local counters) after bbo_count_prepare().  out[30] = per env-step sums over this call
// (not means) of {add/sub, mul, div, sqrt, transcendental, comparisons} per phase; returns the
// env-steps run.
long long bbo_count_flops_replay(int n_envs, int n_steps, double* q, double* v, double* w, int* sc,
                                 const float* actions, const float* table, const double* offsets, const int* terr,
                                 int max_ep, double size_z, double* out, int* overrun) {
  bbo_env_cfg cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.max_ep_steps = 4000;
  cfg.max_allowed_tilt = 20.0;
  cfg.max_wheel_velocity = 10.0;
  cfg.reward_scale = 0.01f;
  cfg.action_reg_coef = -0.0001f;
  cfg.survival_bonus = 0.02f;
  cfg.target_dir[0] = 0.0f;
  cfg.target_dir[1] = 1.0f;
  const size_t HF = (size_t)BBO_HF_N * BBO_HF_N;
  FD* Q = (FD*)calloc((size_t)n_envs * NQ, sizeof(FD));
  FD* V = (FD*)calloc((size_t)n_envs * NV, sizeof(FD));
  FD* W = (FD*)calloc((size_t)n_envs * NV, sizeof(FD));
  int* ep = (int*)calloc((size_t)n_envs, sizeof(int));
  for (size_t i = 0; i < (size_t)n_envs * NQ; i++) Q[i] = FD(q[i]);
  for (size_t i = 0; i < (size_t)n_envs * NV; i++) { V[i] = FD(v[i]); W[i] = FD(w[i]); }
  fc::g = fc::Counts{};
  for (auto& c : fc::ph) c = fc::Counts{};
  fc::cur = 4;
  long long steps = 0;
  for (int e = 0; e < n_envs; e++)
    for (int t = 0; t < n_steps; t++) {
      const int slot = terr[(size_t)e * max_ep + ep[e]];
      const float* a = actions + ((size_t)t * n_envs + e) * 3;
      float obs[15], r, p2[2];
      const int f = bbo_env_step(&cfg, Q + e * NQ, V + e * NV, W + e * NV, sc + e, a, table + (size_t)slot * HF,
                                 FD(size_z), obs, &r, p2, nullptr);
      steps++;
      if (f & 1) {  // auto-reset onto the env's next drawn terrain
        if (ep[e] + 1 < max_ep) ep[e]++; else (*overrun)++;
        const int ns = terr[(size_t)e * max_ep + ep[e]];
        bbo_reset_state(FD(offsets[ns]), Q + e * NQ, V + e * NV, W + e * NV);
        sc[e] = 0;
      }
    }
  fc::phase(4);
  for (int p = 0; p < fc::NPH; p++) {
    const fc::Counts& c = fc::ph[p];
    double* o = out + 6 * p;
    o[0] = (double)c.add; o[1] = (double)c.mul; o[2] = (double)c.div; o[3] = (double)c.sqrt; o[4] = (double)c.trans;
    o[5] = (double)c.cmp;
  }
  for (size_t i = 0; i < (size_t)n_envs * NQ; i++) q[i] = Q[i].v;
  for (size_t i = 0; i < (size_t)n_envs * NV; i++) { v[i] = V[i].v; w[i] = W[i].v; }
  free(Q); free(V); free(W); free(ep);
  return steps;
}

}  // extern "C"
