// bb_solve.h -- team-parallel constrained Newton solve (mj_solNewton, elliptic
// cones) for one env, executed by a team of L lanes of one wavefront.
//
// Minimises  f(a) = 0.5 a'Ma - a'qfs + sum_c s_c(J_c a - aref_c)   over qacc a
// (the primal of MuJoCo's constraint problem; M > 0 so the minimiser is unique
// and any convergent method reproduces it).  Work split inside the team:
//   contact pass    contacts c = tl, tl+L, ...: jar, zone, force, cone Hessian
//   ground terms    6x6 ball-block partials reduced across the team (shuffles)
//   Hessian         entries e = tl, tl+L, ... of the packed 15x15 (LDS)
//   Cholesky        right-looking, column scaling and trailing update in LDS
//   line search     contact-parallel phi'/phi'' partials + team reduction
// Small vectors (a, g, s, Ma) are replicated in every lane's registers; the
// triangular solves and the mass products are computed redundantly per lane.
// With L = 1 (host tests) every loop covers everything and syncs vanish.
#pragma once

#include "bb_physics.h"

namespace bb {

#ifdef BB_SOLVE_STATS
static long g_ls_evals = 0;
static long g_ls_hist[16] = {0};  // line-search evaluations per Newton iteration
static long g_alpha1 = 0;         // Newton iterations whose first evaluation (alpha = 1) was accepted
static int g_stage_iters[4] = {0, 0, 0, 0};  // Newton iterations of each RK stage of the last step
#endif

// Diagnostic build only (-DBB_PHASE_CLOCKS): per-phase s_memtime cycles,
// summed over teams into bb_phase_cycles[] (read back by tools/phase_clocks).
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
extern __device__ unsigned long long bb_phase_cycles[100];
#define PH_DECL unsigned long long ph_t = clock64(), ph_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define PH(k) { unsigned long long n_ = clock64(); ph_acc[k] += n_ - ph_t; ph_t = n_; }
// phases 0-7 -> slots 0-7; 8 (line-search setup) -> 32, 9 (line-search loop) -> 33
#define PH_FLUSH(tm) if ((tm).tl == 0) { for (int k_ = 0; k_ < 8; k_++) atomicAdd(&bb_phase_cycles[k_], ph_acc[k_]); \
                                          atomicAdd(&bb_phase_cycles[32], ph_acc[8]); atomicAdd(&bb_phase_cycles[33], ph_acc[9]); }
// the full kernel's solves (base-tree contacts) separately: phases 0-9 -> slots 80-89
#define PH_FLUSH_BODY(tm) if ((tm).tl == 0) { for (int k_ = 0; k_ < 10; k_++) atomicAdd(&bb_phase_cycles[80 + k_], ph_acc[k_]); }
#elif defined(BB_ISA_MARKS) && defined(__HIP_DEVICE_COMPILE__)
// ISA analysis build: phase boundaries as assembler comments
#define PH_DECL
#define PH(k) asm volatile("; PHASE_MARK " #k);
#define PH_TOP asm volatile("; PHASE_MARK 10");
#define PH_FLUSH(tm)
#define PH_FLUSH_BODY(tm)
#else
#define PH_DECL
#define PH(k)
#define PH_FLUSH(tm)
#define PH_FLUSH_BODY(tm)
#endif
#ifndef PH_TOP
#define PH_TOP
#endif

struct Team {
  int L;   // lanes per env (power of two, <= 64)
  int tl;  // this lane's index inside the team
};

template <typename T>
BB_HD T team_sum(const Team& tm, T v) {
#ifdef __HIP_DEVICE_COMPILE__
  for (int off = tm.L >> 1; off > 0; off >>= 1) v += __shfl_xor(v, off, tm.L);
#else
  (void)tm;
#endif
  return v;
}

BB_HD void team_sync() {
#ifdef __HIP_DEVICE_COMPILE__
#ifdef BB_SYNC_BARRIER
  __syncthreads();
#else
  // orders the wave's LDS traffic across its lanes.  A team lives inside one
  // wave, whose lanes execute together and whose LDS operations complete in
  // order, so a workgroup fence (wait for the wave's LDS operations) and a
  // compiler barrier are enough -- no s_barrier, which in a multi-wave
  // workgroup (relief_multi_kernel) would also wait for the other waves.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
#endif
}

#ifdef __HIPCC__
// bit offset of this lane's team in a 64-bit wave ballot: the team's first lane
// WITHIN THE WAVE.  (threadIdx.x & ~(L-1) is that only in one-wave workgroups;
// in relief_multi_kernel's 4-wave workgroups it reaches 240, a shift past 63.)
__device__ __forceinline__ int team_shift_of(int L) { return (int(threadIdx.x) & 63) & ~(L - 1); }
#endif

// true in every lane of the team if b holds in any of its lanes (team-uniform branch)
BB_HD bool team_any(const Team& tm, bool b) {
#ifdef __HIP_DEVICE_COMPILE__
  const unsigned long long m = __ballot(b);
  const int sh = team_shift_of(tm.L);
  const unsigned long long mask = tm.L >= 64 ? ~0ull : ((1ull << tm.L) - 1);
  return ((m >> sh) & mask) != 0;
#else
  (void)tm;
  return b;
#endif
}

// packed lower-triangle index e -> (i, j), j <= i
BB_HD void tri_unpack(int e, int& i, int& j) {
  int r = (int)((sqrtf(8.f * float(e) + 1.f) - 1.f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= e) r++;
  while (r * (r + 1) / 2 > e) r--;
  i = r;
  j = e - r * (r + 1) / 2;
}

// What mjData holds after the last forward of mj_step (RK stage 4).
template <typename T>
struct StageOut {
  T quat_b[4];   // xquat[base] (normalised)
  T w_world[3];  // cvel[base][0:3]
  T v_com[3];    // cvel[base][3:6] (linear velocity at subtree_com[base])
  T pb[3];       // xpos[base]
  int ng, nb, iters, overflow;
};

// The terrain an env steps on: heightfield (NULL: none), vertical scale and
// its top height max(hfield) * size_z (base-tree geoms above it skip the
// prism search).
template <typename T>
struct TerrainRef {
  const float* hf;
  T size_z, hz;
};

// Per-env working set of one RK step (LDS on the GPU, one per team).
// Phase-local buffers share storage in a union to fit 16 envs per CU.
template <typename T>
struct EnvWork {
  T q0[NQ], v0[NV], vs[NV], as[NV];          // RK4 stage context
  T k1[NV];                                  // stage-1 qacc (stage 4's warm start 2 k3 - k1)
  T qn[NQ], vn[NV], wn[NV];                  // env state and warm start (step kernel: not held in
                                             // registers across the solves)
  T qfs[NV];                                 // smooth force of the current forward
  T vi[NV];                                  // stage velocity (pre-phase; constraint aref rebuilds)
  StageOut<T> so;                            // stage-4 outputs for obs/reward
  Mass<T> M;                                 // mass-matrix blocks
  WheelCon<T> wc[3];                         // ball-wheel contacts
  T g[MAXG * NGF];                           // ball-terrain contacts (compact, GF_*)
  T bc[MAXB_LDS * NBF];                      // base-tree geom contacts 0..MAXB_LDS-1 (compact, BF_*)
  T* bspill;                                 // contacts MAXB_LDS..MAXB-1: this env's HBM block (full kernel)
#ifdef BB_PHASE_CLOCKS
  int dbg_nb;                                // diagnostic build: base-tree contacts summed over the step's forwards
#endif
  Poses<T> P;                                // body poses for the Jacobian rebuilds
  T H[NH];                                   // Hessian / Cholesky factor (packed lower); dense M on the GPU
  union U {
    struct {                                 // forward pre-phase
      Kin<T> k;
      T Iw[3][6];
      T qi[NQ];                              // stage position
    } pre;
    struct {                                 // Hessian assembly
      T cj[3][3][13];                        // C J for each wheel contact
      T wf[3][3];                            // wheel contact forces
      T hg[21];                              // ground contribution to the ball block
    } hes;
  } u;
};

// base-tree contact b: the first MAXB_LDS in LDS, the rest in the env's spill block
template <typename T>
BB_HD T* body_slot(T* bc, T* spill, int b) {
  return b < MAXB_LDS ? bc + b * NBF : spill + (b - MAXB_LDS) * NBF;
}

// Mass-matrix entry (i >= j) from the block representation.
template <typename T>
BB_HD T mass_entry(const Mass<T>& M, int i, int j) {
  if (i < 3) return i == j ? M.mt : T(0);
  if (i < 6) {
    if (j < 3) return M.Mtr[3 * j + (i - 3)];
    const int a = i - 3, b = j - 3;
    return a == b ? M.Mrr[a] : M.Mrr[a + b + 2];  // (1,0)->3, (2,0)->4, (2,1)->5
  }
  if (i < 9) {
    const int w = i - 6;
    if (j < 3) return M.Mth[w][j];
    if (j < 6) return M.Mrh[w][j - 3];
    return j == i ? M.Mhh[w] : T(0);
  }
  if (j < 9) return T(0);
  if (i < 12) return i == j ? M.mB : T(0);
  if (j < 12) return M.MBtr[3 * (j - 9) + (i - 12)];
  return i == j ? M.MBrr[i - 12] : T(0);
}

// position of dof i among wheel w's 13 contact columns, or -1
BB_HD int wheel_pos(int i, int w) { return i < 6 ? i : (i == 6 + w ? 6 : (i >= 9 ? i - 2 : -1)); }

// J_r x for wheel contact w (w may be lane-dependent: the hinge entry is selected)
template <typename T>
BB_HD T wheel_dot(const WheelCon<T>& C, int w, int r, const T* x) {
  const T xh = hinge_sel(w, x);
  T acc = C.J[r][6] * xh;
#pragma unroll
  for (int i = 0; i < 6; i++) acc += C.J[r][i] * x[i];
#pragma unroll
  for (int i = 7; i < 13; i++) acc += C.J[r][i] * x[i + 2];
  return acc;
}

// J_r x over the ball dofs for ground-contact rows J (ground_rows)
template <typename T>
BB_HD T ground_dot(const T (&J)[3][6], int r, const T* x) {
  return J[r][0] * x[9] + J[r][1] * x[10] + J[r][2] * x[11] + J[r][3] * x[12] + J[r][4] * x[13] + J[r][5] * x[14];
}

// Team-parallel right-looking Cholesky in place.  A pivot that roundoff drives
// below eps * (original diagonal) is floored so the direction stays finite;
// descent is enforced by the line search.
template <typename T>
BB_HD void chol_team(T* H, const T* hd, const Team& tm) {
  for (int j = 0; j < NV; j++) {
    team_sync();
    const int rj = j * (j + 1) / 2;
    T s = H[rj + j];
    const T floor_j = pivot_eps<T>() * maxT(hd[j], T(1e-30));
    s = s > floor_j ? s : floor_j;
    const T d = sqrt(s), id = T(1) / d;
    for (int i = j + 1 + tm.tl; i < NV; i += tm.L) H[i * (i + 1) / 2 + j] *= id;
    team_sync();
    if (tm.tl == 0) H[rj + j] = d;
    const int md = NV - 1 - j, cnt = md * (md + 1) / 2;
    for (int t = tm.tl; t < cnt; t += tm.L) {
      int ii, kk;
      tri_unpack(t, ii, kk);
      const int i = j + 1 + ii, k = j + 1 + kk;
      H[i * (i + 1) / 2 + k] -= H[i * (i + 1) / 2 + j] * H[k * (k + 1) / 2 + j];
    }
  }
  team_sync();
}

// One contact along the Newton direction s, in the cone variables of
// mj_constraintUpdate's elliptic zones: U(alpha) = u0 + alpha du with
// U = (mu jar0, f1 jar1, f2 jar2) and jar = J (a + alpha s) - aref.  Prepared
// once per Newton iteration; each line-search evaluation then costs the zone
// tests and the closed-form derivatives of the contact's cost:
//   top     (N >= mu T)            0
//   bottom  (mu N + T <= 0)        1/2 sum_r D_r jar_r^2   -> b0 + alpha b1, b1
//   middle                         1/2 Dm g^2, g = N - mu T -> Dm g g', Dm (g'^2 + g g'')
// with T(alpha) = |U_t(alpha)|, T' = U_t.dU_t / T, T'' = (|dU_t|^2 - T'^2) / T.
// kink: the alpha where T is smallest, if the contact is in the middle zone
// there.  Near it phi' turns by ~Dm g mu |dU_t| within a width of
// T_min / |dU_t| (for a wheel, the axle friction 0.001 of ballbot.xml:90-92
// sets T_min): a near-kink that the line search evaluates before stepping
// across (LineSearch::update); -1 when there is none.
template <typename T>
struct LsTerm {
  T u0[3], du[3], mu, Dm, b0, b1, vv, kink;
  T c0;  // the contact's cost at alpha = 0 in the bottom zone (0.5 sum D_r jar_r^2)
  // phi_c(alpha): the contact's constraint cost (mj_constraintUpdate's zones)
  BB_HD T cost(T alpha) const {
    const T N = u0[0] + alpha * du[0], U1 = u0[1] + alpha * du[1], U2 = u0[2] + alpha * du[2];
    const T Tn = sqrt(U1 * U1 + U2 * U2);
    const bool top = N >= mu * Tn;
    const bool bot = !top && mu * N + Tn <= 0;
    const T g = N - mu * Tn;
    return top ? T(0) : (bot ? c0 + alpha * (b0 + T(0.5) * alpha * b1) : T(0.5) * Dm * g * g);
  }
  BB_HD void prep(const T* j0, const T* x, T mu_, T f1, T f2, const T* D, T Dm_) {
    mu = mu_;
    Dm = Dm_;
    u0[0] = mu * j0[0]; u0[1] = f1 * j0[1]; u0[2] = f2 * j0[2];
    du[0] = mu * x[0]; du[1] = f1 * x[1]; du[2] = f2 * x[2];
    b0 = D[0] * j0[0] * x[0] + D[1] * j0[1] * x[1] + D[2] * j0[2] * x[2];
    b1 = D[0] * x[0] * x[0] + D[1] * x[1] * x[1] + D[2] * x[2] * x[2];
    c0 = T(0.5) * (D[0] * j0[0] * j0[0] + D[1] * j0[1] * j0[1] + D[2] * j0[2] * j0[2]);
    vv = du[1] * du[1] + du[2] * du[2];
    kink = T(-1);
    if (vv > 0) {
      const T ak = -(u0[1] * du[1] + u0[2] * du[2]) / vv;
      const T N = u0[0] + ak * du[0], U1 = u0[1] + ak * du[1], U2 = u0[2] + ak * du[2];
      const T Tn = sqrt(U1 * U1 + U2 * U2);
      if (ak > 0 && N < mu * Tn && mu * N + Tn > 0) kink = ak;
    }
  }
  BB_HD void none() {
    u0[0] = u0[1] = u0[2] = du[0] = du[1] = du[2] = T(0);
    u0[0] = T(1);  // separated: top zone at every alpha
    mu = Dm = b0 = b1 = vv = c0 = T(0);
    kink = T(-1);
  }
  // adds phi_c'(alpha), phi_c''(alpha) and a magnitude bound of the terms of phi_c'
  BB_HD void eval(T alpha, T& d1, T& d2, T& dm) const {
    const T N = u0[0] + alpha * du[0], U1 = u0[1] + alpha * du[1], U2 = u0[2] + alpha * du[2];
    const T t2 = U1 * U1 + U2 * U2;
    const T rt = t2 > 0 ? rsqrt_ls(t2) : T(0);
    const T Tn = t2 * rt;
    const bool top = (N >= mu * Tn) | ((Tn <= 0) & (N >= 0));   // bitwise: selects, not branches
    const bool bot = !top & ((mu * N + Tn <= 0) | ((Tn <= 0) & (N < 0)));
    const T g = N - mu * Tn;
    const T tp = (U1 * du[1] + U2 * du[2]) * rt;
    const T gp = du[0] - mu * tp;
    const T tpp = (vv - tp * tp) * rt;
    const T Dg = Dm * g;
    const T m1 = Dg * gp, m2 = Dm * gp * gp - mu * Dg * tpp;
    const T q1 = b0 + alpha * b1;
    d1 += top ? T(0) : (bot ? q1 : m1);
    d2 += top ? T(0) : (bot ? b1 : m2);
    dm += top ? T(0) : (bot ? fabs(b0) + fabs(alpha * b1) : fabs(Dg) * (fabs(du[0]) + mu * fabs(tp)));
  }
};

// One update of the exact line search on phi'(alpha) (phi convex, phi'
// continuous and nondecreasing): the evaluation (alpha, d1 = phi', d2 = phi'')
// tightens the bracket [lo, hi] and picks the next alpha.  1-D Newton from the
// latest point while it lands inside the bracket and its step is less than
// half the step before the last one (the progress test of a safeguarded
// Newton, as in rtsafe); otherwise Illinois false position on the bracket.
// The failures this catches: a stiff drive-direction row (R scaled by
// (0.001/1)^2, ballbot.xml:90-92) changes cone zone between lo and hi, so
// phi'' jumps by ~1e6 there, and Newton steps from the smooth parts either
// overshoot back and forth across it (a 2-cycle that keeps the bracket for
// up to ls_maxiter evaluations) or creep towards it.
//
// Kinks (LsTerm::kink): a step that would cross a contact's near-kink stops
// at it instead; the bracket then closes on the kink from either side in a
// few evaluations.
template <typename T>
struct LineSearch {
  T lo, dlo, hi, dhi, alpha, flo, fhi, prev, dx, dxold;
  int side, same;
  BB_HD void init(T d0) {
    lo = 0; dlo = d0; hi = -1; dhi = 0; alpha = 1; flo = d0; fhi = 0; prev = 0;
    dx = dxold = T(1e30);
    side = 0; same = 0;
  }
  // is the kink k strictly between the last evaluated point and the proposed
  // one, and inside the bracket?
  BB_HD bool crosses(T k) const {
    const bool between = alpha > prev ? (k > prev && k < alpha) : (k < prev && k > alpha);
    return between && k > lo && (hi < 0 || k < hi);
  }
  // select-only (no branches): the lanes of a team agree, the teams of a wave
  // do not, and divergent branches would run every path with exec masks
  BB_HD void update(T d1, T d2) {
    prev = alpha;
    const bool neg = d1 < 0;
    const int sd = neg ? -1 : 1;
    same = sd == side ? same + 1 : 0;
    side = sd;
    const bool rep = same > 0;
    const T hlo = (!neg & rep) ? T(0.5) : T(1);             // Illinois: halve the stale end's weight
    const T hhi = (neg & rep & (hi >= 0)) ? T(0.5) : T(1);
    lo = neg ? alpha : lo;
    dlo = neg ? d1 : dlo;
    flo = neg ? d1 : flo * hlo;
    hi = neg ? hi : alpha;
    dhi = neg ? dhi : d1;
    fhi = neg ? fhi * hhi : d1;
    const T an_n = alpha - div_ls(d1, maxT(d2, T(1e-30)));  // Newton from the latest point
    const T fp = lo - div_ls(flo * (hi - lo), fhi - flo);   // false position (bracket only)
    const T an_f = ((fp > lo) & (fp < hi)) ? fp : T(0.5) * (lo + hi);
    const T an_o = an_n > lo ? an_n : (lo > 0 ? 2 * lo : T(1));  // no upper end yet
    const bool newton = (an_n > lo) & (an_n < hi) & (fabs(an_n - alpha) <= T(0.5) * dxold);
    const T an = hi < 0 ? an_o : (newton ? an_n : an_f);
    dxold = dx;
    dx = fabs(an - alpha);
    alpha = an;
  }
  // the step was shortened to a kink
  BB_HD void snap(T k) {
    alpha = k;
    dx = fabs(k - prev);
  }
  // an unconverged search falls back to the last point with phi' < 0 (a
  // guaranteed decrease for convex phi)
  BB_HD T fallback() const { return lo > 0 ? lo : (hi > 0 ? hi * dlo / (dlo - dhi) : T(0)); }
};

// Newton on f(a) (mj_solNewton).  a: warm start in, qacc out (replicated in
// every lane of the team).  Returns the iteration count (team-uniform).
// Host / reference path (tests/hostcheck): wheel and ball-hfield contacts
// only; the GPU solve (bb_team16.h) also handles the base-tree contacts.
template <typename T>
BB_HD int solve_team(const ModelT<T>& m, EnvWork<T>& W, const T* qfs, int ng, T* a, const Team& tm) {
  const Mass<T>& M = W.M;
  PH_DECL
  const T mu_w = m.fr_wheel[0], f1w = m.fr_wheel[0], f2w = m.fr_wheel[1];
  const int nc = 3 + ng;
  T hd[NV];  // Hessian diagonal before factorisation (pivot floor)
  int it = 0;
  for (; it < m.maxiter; it++) {
    team_sync();
    // ---- (1) contact pass: forces and cone Hessians, contact-parallel
    T Hg[21], gg[6];
#pragma unroll
    for (int i = 0; i < 21; i++) Hg[i] = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) gg[i] = 0;
    for (int c = tm.tl; c < nc; c += tm.L) {
      if (c < 3) {
        const WheelCon<T>& C = W.wc[c];
        T jar[3], f[3], Cc[6];
#pragma unroll
        for (int r = 0; r < 3; r++) jar[r] = wheel_dot(C, c, r, a) - C.aref[r];
        T Dw[3] = {C.D[0], C.D[1], C.D[2]};
        cone_eval(jar, mu_w, f1w, f2w, Dw, f, Cc);
#pragma unroll
        for (int r = 0; r < 3; r++) W.u.hes.wf[c][r] = f[r];
        for (int i = 0; i < 13; i++) {
          const T j0 = C.J[0][i], j1 = C.J[1][i], j2 = C.J[2][i];
          W.u.hes.cj[c][0][i] = Cc[0] * j0 + Cc[3] * j1 + Cc[4] * j2;
          W.u.hes.cj[c][1][i] = Cc[3] * j0 + Cc[1] * j1 + Cc[5] * j2;
          W.u.hes.cj[c][2][i] = Cc[4] * j0 + Cc[5] * j1 + Cc[2] * j2;
        }
      } else {
        const T* gc = W.g + (c - 3) * NGF;
        T J[3][6], ar[3], D;
        ground_contact(m, gc, W.P.RB, W.vi, J, ar, D);
        T jar[3];
#pragma unroll
        for (int r = 0; r < 3; r++) jar[r] = ground_dot(J, r, a) - ar[r];
        T Dv[3] = {D, D, D}, f[3], Cc[6];
        cone_eval(jar, T(1), T(1), T(1), Dv, f, Cc);
        T w[3][6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
          gg[i] -= J[0][i] * f[0] + J[1][i] * f[1] + J[2][i] * f[2];
          w[0][i] = Cc[0] * J[0][i] + Cc[3] * J[1][i] + Cc[4] * J[2][i];
          w[1][i] = Cc[3] * J[0][i] + Cc[1] * J[1][i] + Cc[5] * J[2][i];
          w[2][i] = Cc[4] * J[0][i] + Cc[5] * J[1][i] + Cc[2] * J[2][i];
        }
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
          for (int j = 0; j <= i; j++) Hg[i * (i + 1) / 2 + j] += J[0][i] * w[0][j] + J[1][i] * w[1][j] + J[2][i] * w[2][j];
      }
    }
    PH(0)
    // ---- (2) reduce the ground partials across the team
#pragma unroll
    for (int i = 0; i < 21; i++) Hg[i] = team_sum(tm, Hg[i]);
#pragma unroll
    for (int i = 0; i < 6; i++) gg[i] = team_sum(tm, gg[i]);
    if (tm.tl == 0) {
#pragma unroll
      for (int i = 0; i < 21; i++) W.u.hes.hg[i] = Hg[i];
    }
    team_sync();
    PH(1)
    // ---- (3) gradient, replicated: g = M a - qfs - sum_c J_c' f_c
    T g[NV], Ma[NV];
    mass_mul(M, a, Ma);
#pragma unroll
    for (int i = 0; i < NV; i++) g[i] = Ma[i] - qfs[i];
#pragma unroll
    for (int i = 0; i < 6; i++) g[9 + i] += gg[i];
#pragma unroll
    for (int w = 0; w < 3; w++) {
      const T f0 = W.u.hes.wf[w][0], f1 = W.u.hes.wf[w][1], f2 = W.u.hes.wf[w][2];
      const WheelCon<T>& C = W.wc[w];
#pragma unroll
      for (int i = 0; i < 13; i++) g[wheel_col(i, w)] -= C.J[0][i] * f0 + C.J[1][i] * f1 + C.J[2][i] * f2;
    }
    T gn = 0;
#pragma unroll
    for (int i = 0; i < NV; i++) gn += g[i] * g[i];
#ifdef BB_SOLVE_TRACE
    printf("it %d |g| %.3e\n", it, double(m.scale * sqrt(gn)));
#endif
    // MuJoCo's gradient stop (mj_solPrimal: scale * ||grad|| < tolerance after an
    // iteration; the first iteration always runs)
    if (it > 0 && m.scale * sqrt(gn) < m.tol) break;
    PH(2)
    // ---- (4) Hessian entries, entry-parallel
    for (int e = tm.tl; e < NH; e += tm.L) {
      int i, j;
      tri_unpack(e, i, j);
      T h = mass_entry(M, i, j);
#pragma unroll
      for (int w = 0; w < 3; w++) {
        const int pi = wheel_pos(i, w), pj = wheel_pos(j, w);
        if (pi >= 0 && pj >= 0) {
          const WheelCon<T>& C = W.wc[w];
          h += C.J[0][pi] * W.u.hes.cj[w][0][pj] + C.J[1][pi] * W.u.hes.cj[w][1][pj] +
               C.J[2][pi] * W.u.hes.cj[w][2][pj];
        }
      }
      if (j >= 9) {
        const int a9 = i - 9, b9 = j - 9;
        h += W.u.hes.hg[a9 * (a9 + 1) / 2 + b9];
      }
      W.H[e] = h;
      if (i == j) hd[i] = h;
    }
    PH(3)
    // ---- (5) factorise, Newton direction (replicated triangular solves)
    chol_team(W.H, hd, tm);
    PH(4)
    T s[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) s[i] = -g[i];
    chol_solve_packed(W.H, s);
    T d0 = 0;
    bool fin = true;
#pragma unroll
    for (int i = 0; i < NV; i++) { fin = fin && isfinite(s[i]); d0 += s[i] * g[i]; }
    if (!fin || !(d0 < 0)) {
      // roundoff-indefinite Hessian (fp32): diagonal Newton fallback
      d0 = 0;
#pragma unroll
      for (int i = 0; i < NV; i++) {
        const T hii = mass_entry(M, i, i);
        s[i] = -g[i] / maxT(hii, T(1e-30));
        d0 += s[i] * g[i];
      }
      if (!(d0 < 0)) break;
    }
    PH(5)
    // ---- (6) exact line search on phi(alpha) = f(a + alpha s)
    T Ms[NV];
    mass_mul(M, s, Ms);
    T sMs = 0, gs = 0;
#pragma unroll
    for (int i = 0; i < NV; i++) { sMs += s[i] * Ms[i]; gs += s[i] * (Ma[i] - qfs[i]); }
    LsTerm<T> lst[3 + MAXG];  // line-search terms (host / reference path: plenty of stack)
    const T kdw = T(1) / (mu_w * mu_w * (1 + mu_w * mu_w));
    for (int c = tm.tl; c < nc; c += tm.L) {
      T j0[3], x[3];
      if (c < 3) {
        const WheelCon<T>& C = W.wc[c];
#pragma unroll
        for (int r = 0; r < 3; r++) { j0[r] = wheel_dot(C, c, r, a) - C.aref[r]; x[r] = wheel_dot(C, c, r, s); }
        lst[c].prep(j0, x, mu_w, f1w, f2w, C.D, C.D[0] * kdw);
      } else {
        const T* gc = W.g + (c - 3) * NGF;
        T J[3][6], ar[3], D;
        ground_contact(m, gc, W.P.RB, W.vi, J, ar, D);
#pragma unroll
        for (int r = 0; r < 3; r++) { j0[r] = ground_dot(J, r, a) - ar[r]; x[r] = ground_dot(J, r, s); }
        const T Dv[3] = {D, D, D};
        lst[c].prep(j0, x, T(1), T(1), T(1), Dv, D * T(0.5));
      }
    }
    // exact line search from the full step (LineSearch)
    LineSearch<T> lsr;
    lsr.init(d0);
    const T& alpha = lsr.alpha;
    bool ls_ok = false;
    for (int ls = 1; ls <= m.ls_maxiter; ls++) {
#ifdef BB_SOLVE_STATS
      g_ls_evals++;
#endif
      T d1p = 0, d2p = 0, dmp = 0;
      for (int c = tm.tl; c < nc; c += tm.L) lst[c].eval(alpha, d1p, d2p, dmp);
      const T d1 = gs + alpha * sMs + team_sum(tm, d1p);
      const T d2 = sMs + team_sum(tm, d2p);
      const T dmag = fabs(gs) + fabs(alpha * sMs) + team_sum(tm, dmp);
#ifdef BB_LS_TRACE
      printf("    ls %d alpha %.17g d1 %.6e d2 %.6e d0 %.6e", ls, double(alpha), double(d1), double(d2), double(d0));
      if (ls == 1) {
        printf(" kinks");
        for (int c = 0; c < nc; c++) if (lst[c].kink > 0) printf(" %d:%.4g", c, double(lst[c].kink));
      }
      printf("\n");
#endif
      if (fabs(d1) <= m.ls_tol * fabs(d0) || fabs(d1) <= T(32) * eps_of<T>() * dmag) {
        ls_ok = true;
#ifdef BB_SOLVE_STATS
        g_ls_hist[ls < 15 ? ls : 15]++;
        if (ls == 1) g_alpha1++;
#endif
        break;
      }
      if (!(d1 == d1)) break;
      lsr.update(d1, d2);
#ifndef BB_NO_KINK
      {
        // the crossed kink nearest the last evaluated point
        const bool up = lsr.alpha > lsr.prev;
        T kn = T(-1);
        for (int c = 0; c < nc; c++)
          if (lsr.crosses(lst[c].kink) && (kn < 0 || (up ? lst[c].kink < kn : lst[c].kink > kn))) kn = lst[c].kink;
        if (kn > 0) lsr.snap(kn);
      }
#endif
    }
    if (!ls_ok) lsr.alpha = lsr.fallback();
#ifdef BB_SOLVE_TRACE
    printf("   d0 %.3e alpha %.3e ls_ok %d lo %.3e hi %.3e dlo %.3e dhi %.3e\n", double(d0), double(alpha), int(ls_ok),
           double(lsr.lo), double(lsr.hi), double(lsr.dlo), double(lsr.dhi));
#endif
    if (!(alpha > 0)) break;
    // the cost change of the step, closed form on the line: the Gauss term
    // alpha (s'(Ma - qfs)) + alpha^2 s'Ms / 2, plus each contact's phi_c(alpha) - phi_c(0)
    T dc = 0;
    for (int c = tm.tl; c < nc; c += tm.L) dc += lst[c].cost(alpha) - lst[c].cost(T(0));
    const T dcost = alpha * (gs + T(0.5) * alpha * sMs) + team_sum(tm, dc);
    T sn = 0, an2 = 0;
#pragma unroll
    for (int i = 0; i < NV; i++) { a[i] += alpha * s[i]; sn += s[i] * s[i]; an2 += a[i] * a[i]; }
    PH(6)
    if (alpha * alpha * sn <= T(1e-30) + m.step_rel2 * (1 + an2)) { it++; break; }
    // MuJoCo's improvement stop (mj_solPrimal: scale * (oldcost - cost) < tolerance)
    if (-m.scale * dcost < m.tol) { it++; break; }
  }
  PH(7)
  PH_FLUSH(tm)
  return it;
}

}  // namespace bb
