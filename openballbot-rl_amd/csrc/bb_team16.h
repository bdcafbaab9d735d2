// bb_team16.h -- the constraint solve of bb_solve.h mapped onto one 16-lane
// DPP row of a gfx950 wavefront (device only).
//
// A team of 16 lanes == one DPP row, so every cross-lane step is a DPP move
// (1 VALU op, no LDS round trip):
//   team sum      row_mirror, row_half_mirror, quad_perm [2,3,0,1], [1,0,3,2]
//                 (every lane ends with the bit-identical total)
//   broadcast     row_newbcast:j (lane j of the row to all 16)
// Work split per Newton iteration:
//   contact pass  lane c owns contact c (c, c+16): cone force / Hessian; its
//                 -J'f and ground-block C-weighted J'J partials are team-summed
//   Hessian       lane i owns ROW i of H in registers: dense M row (LDS, built
//                 once per forward) + wheel blocks J_w' (C J)_w + ground block
//   Cholesky      right-looking on the register rows; column j scaled by the
//                 broadcast pivot, trailing update with broadcast L_kj
//   solves        forward: column sweep with broadcasts; backward: one team
//                 sum per unknown (lane k holds L_ki)
//   line search   contact-parallel phi'/phi'' partials + 3 team sums
// The arithmetic per quantity is the same as bb_solve.h:solve_team (which the
// host tests run); only the distribution over lanes differs.
#pragma once

#include <type_traits>

#include "bb_bodycon.h"
#include "bb_solve.h"

namespace bb {
#ifdef __HIP_DEVICE_COMPILE__
namespace t16 {

constexpr int L = 16;

// every pattern used here reads a valid lane of the same row, so no "old"
// value is needed (mov_dpp: no register initialisation before each move)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// doubles: row_newbcast (0x150 + j) is the one DPP control gfx950 applies to a
// 64-bit move (v_mov_b64_dpp, DPP64); the other patterns move two 32-bit halves
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  if constexpr (CTRL >= 0x150 && CTRL <= 0x15F)
    return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(v), CTRL, 0xF, 0xF, true));
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// sum over the 16 lanes of the row; identical bits in every lane
template <typename T>
__device__ __forceinline__ T tsum(T v) {
  v += dpp<0x140>(v);  // row_mirror       i <-> 15-i
  v += dpp<0x141>(v);  // row_half_mirror  i <-> 7-i within each half
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}

// tsum of N values at once, stage by stage: each value's sums are tsum's, bit for bit, but the N
// DPP chains are interleaved, so no stage waits on the previous one's result
template <int N, typename T>
__device__ __forceinline__ void tsum_n(T (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp<0x140>(x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp<0x141>(x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp<0x4E>(x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp<0xB1>(x[i]);
}

// minimum over the 16 lanes of the row (exact: identical in every lane)
template <typename T>
__device__ __forceinline__ T tmin(T v) {
  v = fmin(v, dpp<0x140>(v));  // v_min (no NaNs here: kinks or the 1e30 sentinel)
  v = fmin(v, dpp<0x141>(v));
  v = fmin(v, dpp<0x4E>(v));
  v = fmin(v, dpp<0xB1>(v));
  return v;
}

// lane J's value to the whole row
template <int J, typename T>
__device__ __forceinline__ T bcast(T v) {
  return dpp<0x150 + J>(v);
}

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (N > 0) {
    static_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}

// cone_eval (bb_physics.h) without branches: the three zones are computed and
// selected, so lanes of a team in different zones do not serialise.
template <typename T>
__device__ __forceinline__ void cone_sel(const T* jar, T mu, T f1, T f2, const T* D, T Dm, T* force, T* C) {
  const T U0 = jar[0] * mu, U1 = jar[1] * f1, U2 = jar[2] * f2;
  const T t2 = U1 * U1 + U2 * U2;
  const T rt = t2 > 0 ? rsqrt(t2) : T(0);
  const T N = U0, Tn = t2 * rt;  // sqrt(t2) via the reciprocal root the Hessian needs anyway
  const bool top = N >= mu * Tn || (Tn <= 0 && N >= 0);
  const bool bot = !top && (mu * N + Tn <= 0 || (Tn <= 0 && N < 0));
  const T g = N - mu * Tn;  // Dm = D0 / (mu^2 (1 + mu^2)) from cone_params
  const T iT = Tn > 0 ? rt : T(1);
  const T gr1 = -mu * f1 * U1 * iT, gr2 = -mu * f2 * U2 * iT;
  const T sc = -Dm * g;
  const T k = Dm * g * (-mu) * iT, iT2 = iT * iT;
  T fm[3] = {sc * mu, sc * gr1, sc * gr2};
  T cm[6] = {Dm * mu * mu, Dm * gr1 * gr1 + k * f1 * f1 * (T(1) - U1 * U1 * iT2),
             Dm * gr2 * gr2 + k * f2 * f2 * (T(1) - U2 * U2 * iT2), Dm * mu * gr1, Dm * mu * gr2,
             Dm * gr1 * gr2 - k * f1 * f2 * U1 * U2 * iT2};
#pragma unroll
  for (int r = 0; r < 3; r++) force[r] = top ? T(0) : (bot ? -D[r] * jar[r] : fm[r]);
#pragma unroll
  for (int r = 0; r < 6; r++) C[r] = top ? T(0) : (bot ? (r < 3 ? D[r] : T(0)) : cm[r]);
}

// which wheel dof a 13-column contact Jacobian's column q maps to (-1: none)
__device__ __forceinline__ int col_dof(int q, int hinge) { return q < 6 ? q : (q == 6 ? (hinge >= 0 ? 6 + hinge : -1) : q + 2); }

// 1/sqrt(x) for the Cholesky pivots: the hardware estimate and one
// second-order correction r (1 + e/2 + 3e^2/8), e = 1 - x r^2 (the device
// library's sequence without its inf/zero class check: the pivots are
// floored, so x > 0 and finite); the pivot chain is the factorisation's
// critical path
template <typename T>
__device__ __forceinline__ T rsqrt_piv(T x) {
  if constexpr (sizeof(T) == 8) {
    const double r = __builtin_amdgcn_rsq(x);
    const double e = fma(-x * r, r, 1.0);
    return fma(r * e, fma(e, 0.375, 0.5), r);
  } else {
    return __builtin_amdgcn_rsqf(x);
  }
}

// Cholesky of the register-distributed H (lane i holds row h[0..14]); on exit
// lane i holds L_ik (k < i) in h[k] and every lane holds diag[] = 1 / L_jj.
// Entries right of a lane's diagonal (the upper triangle) are updated too,
// without a select: they are never read, by the factorisation or the solves.
template <typename T>
__device__ __forceinline__ void chol_rows(T (&h)[NV], T hdi, T (&diag)[NV], int tl) {
  static_for<NV>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    T piv = bcast<j>(h[j]);
    const T hdj = bcast<j>(hdi);
    const T fl = pivot_eps<T>() * maxT(hdj, T(1e-30));
    piv = fmax(piv, fl);  // one v_max on the pivot chain (piv is finite or the direction is rejected)
    const T id = rsqrt_piv(piv);  // 1 / L_jj in one reciprocal square root (no sqrt + divide chain)
    diag[j] = id;  // inverse pivot: the solves multiply
    h[j] *= id;
    static_for<NV - 1 - j>([&](auto kc) {
      constexpr int k = j + 1 + decltype(kc)::value;
      const T lkj = bcast<k>(h[j]);
      h[k] -= h[j] * lkj;
    });
  });
}

// s = -(L L')^-1 g with L distributed by rows (lane i: L_i,0..i-1 in h[]);
// lane i supplies g_i (gown) and gets the whole s (replicated) plus its own
// component s_i (sown); lanes >= NV get sown = 0.
//   forward   L y = -g, column sweep: lane j's right-hand side broadcast, every
//             later row updates its own
//   backward  L' s = y, column sweep over L' after a transpose through LDS
//             (scr: >= NV (NV - 1) / 2 elements of team scratch): lane k holds
//             column k of L, so s_i needs one broadcast instead of a team sum
template <typename T>
__device__ __forceinline__ void chol_solve_rows(const T (&h)[NV], const T (&diag)[NV], T gown, T (&s)[NV], T& sown,
                                                int tl, T* scr) {
  T b = tl < NV ? -gown : T(0);
  T z = 0;  // y of this lane's row
  static_for<NV>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const T yj = bcast<j>(b) * diag[j];
    z = tl == j ? yj : z;
    b -= h[j] * yj;  // rows <= j no longer read their right-hand side
  });
  // strictly lower L, packed by rows (row i at i (i - 1) / 2)
  if (tl < NV) {
    static_for<NV - 1>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if (k < tl) scr[tl * (tl - 1) / 2 + k] = h[k];
    });
  }
  team_sync();
  T Lc[NV];  // Lc[i] = L_i,tl below the diagonal, else 0
  static_for<NV>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    Lc[i] = (i > tl) ? scr[i * (i - 1) / 2 + tl] : T(0);
  });
  T own = 0;
  static_for<NV>([&](auto ic) {
    constexpr int i = NV - 1 - decltype(ic)::value;
    const T si = bcast<i>(z) * diag[i];
    s[i] = si;
    z -= Lc[i] * si;
    own = tl == i ? si : own;
  });
  sown = own;
}

// stored base-tree contact b into registers: LDS slot or the env's HBM spill
// block, each through its own address space (a pointer select between the two
// compiles to generic flat loads)
template <typename T>
__device__ __forceinline__ void body_load(const EnvWork<T>& W, int b, T (&o)[NBF]) {
  if (b < MAXB_LDS) {
    const T* p = W.bc + b * NBF;
#pragma unroll
    for (int i = 0; i < NBF; i++) o[i] = p[i];
  } else {
    const T* p = W.bspill + (b - MAXB_LDS) * NBF;
#pragma unroll
    for (int i = 0; i < NBF; i++) o[i] = p[i];
  }
}

// line-search terms of contact c: jar(0) = J a - aref, J s and the contact's
// D (isotropic contacts) -- zeros when c >= nc
template <bool BODY, typename T>
__device__ __forceinline__ void ls_terms(const ModelT<T>& m, const EnvWork<T>& W, int c, int ng, int nc, const T* a,
                                         const T* s, T (&c6)[6], T& D) {
#pragma unroll
  for (int r = 0; r < 6; r++) c6[r] = 0;
  D = 0;
  if (c >= nc) return;
  if (c < 3) {
    const WheelCon<T>& C = W.wc[c];
#pragma unroll
    for (int r = 0; r < 3; r++) { c6[r] = wheel_dot(C, c, r, a) - C.aref[r]; c6[3 + r] = wheel_dot(C, c, r, s); }
  } else if (c < 3 + ng) {
    T J[3][6], ar[3];
    ground_contact(m, W.g + (c - 3) * NGF, W.P.RB, W.vi, J, ar, D);
#pragma unroll
    for (int r = 0; r < 3; r++) { c6[r] = ground_dot(J, r, a) - ar[r]; c6[3 + r] = ground_dot(J, r, s); }
  } else if constexpr (BODY) {
    T bcv[NBF];
    body_load(W, c - 3 - ng, bcv);
    body_ls_terms(m, bcv, W.P, W.vi, a, s, c6, D);
  }
}

// LsTerm (bb_solve.h) of contact c for the line search along s; an inert
// term when c >= nc
template <bool BODY, typename T>
__device__ __forceinline__ void ls_term(const ModelT<T>& m, const EnvWork<T>& W, int c, int ng, int nc, const T* a,
                                        const T* s, T kdw, LsTerm<T>& lt) {
  T c6[6], Dc;
  ls_terms<BODY>(m, W, c, ng, nc, a, s, c6, Dc);
  if (c >= nc) {
    lt.none();
    return;
  }
  const bool wheel = c < 3;
  const T D[3] = {wheel ? W.wc[c].D[0] : Dc, wheel ? W.wc[c].D[1] : Dc, wheel ? W.wc[c].D[2] : Dc};
  const T mu = wheel ? m.fr_wheel[0] : T(1), f1 = wheel ? m.fr_wheel[0] : T(1), f2 = wheel ? m.fr_wheel[1] : T(1);
  lt.prep(c6, c6 + 3, mu, f1, f2, D, D[0] * (wheel ? kdw : T(0.5)));  // Dm = D0 / (mu^2 (1 + mu^2))
}

// ---------------------------------------------------------------------------
// Newton on f(a) (mj_solNewton), a replicated in every lane of the row; W.H
// holds the dense mass matrix (packed lower) for this forward, W.qfs the
// smooth force.  The host reference (bb_solve.h:solve_team) runs the same
// iteration serially.  Work split over the 16 lanes:
//   per forward    fast kernel: lane 3+c builds ball-terrain contact c's
//                  Jacobian, aref and D once (ground_setup) into LDS for
//                  c < GC_LDS (the BODY-only W.bc region and the mass blocks,
//                  dead during the solve); later contacts (rare: more than 13)
//                  and the full kernel's rebuild them per use
//   contact pass   wheel lanes publish C J and f (LDS); ground lanes add their
//                  ball-block gradient and C-weighted J'J partials; base-tree
//                  contacts (full kernel) are rebuilt by one lane each and
//                  broadcast (DPP) so that every lane adds its own Hessian row
//                  and gradient entry
//   gradient       lane i: g_i = (M a)_i - qfs_i - sum_w J_w[:,i]' f_w from its
//                  dense M row and the wheel data, plus the team-summed
//                  ball-block ground part: 6 + 21 team sums (all-replicated
//                  gradient: 15 + 21)
//   line search    s'M s and s'(M a - qfs) from the rows (team sums, no
//                  replicated mass products); each contact term from the
//                  contact pass's jar and the stored Jacobian
constexpr int GC_LDS = 13;  // ball-terrain contacts with an LDS Jacobian (one contact per lane: 3 + 13 = 16)
static_assert(GC_LDS * 18 <= MAXB_LDS * NBF, "ground Jacobians do not fit W.bc");

// aref[3], D of ground contact c (c < GC_LDS), in the mass-block storage
template <typename T>
__device__ __forceinline__ T* ground_ad(EnvWork<T>& W, int c) {
  static_assert(sizeof(Mass<T>) >= GC_LDS * 4 * sizeof(T), "ground aref/D do not fit the mass blocks");
  return reinterpret_cast<T*>(&W.M) + 4 * c;
}

// lane 3 + c: ground contact c's Jacobian rows, aref and D, once per forward
// (they depend on the stage state only).  W.P and W.vi must be set, and the
// mass blocks must be consumed (mass_dense_team) before.
template <typename T>
__device__ __forceinline__ void ground_setup(const ModelT<T>& m, EnvWork<T>& W, int ng, int tl) {
  const int c = tl - 3;
  if (c >= 0 && c < ng && c < GC_LDS) {
    T J[3][6], ar[3], D;
    ground_contact(m, W.g + c * NGF, W.P.RB, W.vi, J, ar, D);
    T* o = W.bc + c * 18;
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int i = 0; i < 6; i++) o[6 * r + i] = J[r][i];
    T* ad = ground_ad(W, c);
#pragma unroll
    for (int r = 0; r < 3; r++) ad[r] = ar[r];
    ad[3] = D;
  }
}

// ground contact c's Jacobian, aref and D: stored (fast kernel), or rebuilt
// past GC_LDS and in the full kernel (its W.bc holds the base-tree contacts)
template <bool BODY, typename T>
__device__ __forceinline__ void ground_get(const ModelT<T>& m, EnvWork<T>& W, int c, T (&J)[3][6], T (&ar)[3], T& D) {
  if (!BODY && c < GC_LDS) {
    const T* o = W.bc + c * 18;
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int i = 0; i < 6; i++) J[r][i] = o[6 * r + i];
    const T* ad = ground_ad(W, c);
#pragma unroll
    for (int r = 0; r < 3; r++) ar[r] = ad[r];
    D = ad[3];
  } else {
    ground_contact(m, W.g + c * NGF, W.P.RB, W.vi, J, ar, D);
  }
}

template <bool BODY, typename T>
__device__ int solve16(const ModelT<T>& m, EnvWork<T>& W, int ng, int nb, T* a, int tl) {
  if constexpr (!BODY) nb = 0;
  const int ngc = 3 + ng;    // wheel and ball-terrain contacts
  const int nc = ngc + nb;   // + base-tree contacts
  const bool rowl = tl < NV;
  const int row = rowl ? tl : NV - 1;
  const T muw = m.fr_wheel[0];
  const T kdw = T(1) / (muw * muw * (1 + muw * muw));
  const T qfs_i = W.qfs[row];
  const int gcol = row - 9;  // this row's ball dof (rows 9..14), else < 0
  // the wheels' f and C (packed C[6], f[3] each) go through LDS (the wf + hg
  // scratch).  Publishing the ball-terrain contacts' the same way for the
  // ball-row owners was measured and dropped: the per-contact LDS loop on the
  // row lanes exposes its latency (flat 0.808 ms/step against 0.666 with the
  // ball-block team sums)
  static_assert(offsetof(typename EnvWork<T>::U, hes.hg) == offsetof(typename EnvWork<T>::U, hes.wf) + 9 * sizeof(T),
                "wheel f/C scratch needs wf and hg adjacent");
  T* const wCf = &W.u.hes.wf[0][0];
  const bool gsum = ng > 0;  // team-uniform
#ifdef BB_HROW_REG
  // this lane's row of the dense mass matrix, held in registers across the Newton
  // iterations (W.H does not change during the solve) instead of re-read from LDS
  T hM[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) hM[k] = W.H[hidx(row, k)];
#define BB_HROW(k) hM[k]
#else
#define BB_HROW(k) W.H[hidx(row, k)]
#endif
  PH_DECL
  int it = 0;
  for (; it < m.maxiter; it++) {
    team_sync();
    PH_TOP
    // the lane index as the sweeps see it, redefined each iteration: otherwise the compiler hoists
    // the fifteen (lane == j) masks out of the Newton loop, keeps them in SGPR pairs and spills
    // them to VGPR lanes, and every use costs two v_readlane and a hazard wait (flat -1.2%)
    int tlx = tl;
    asm volatile("" : "+v"(tlx));
    // ---- (1) contact pass, contact-parallel (c = tl, tl + 16, ...): the
    // wheels' cone force f and Hessian C (3x3, packed) into LDS for the row
    // owners; ball-terrain contacts add ball-block gradient and C-weighted J'J
    // partials for team sums
    T gg[6], Hg[21];
#pragma unroll
    for (int i = 0; i < 6; i++) gg[i] = 0;
#pragma unroll
    for (int i = 0; i < 21; i++) Hg[i] = 0;
    T jar0[3] = {0, 0, 0};  // this lane's first contact, kept for the line search
#ifdef BB_EXP_DUP_CPASS  // timing experiment: the wheel / ball-terrain contact pass twice
    for (int rep = 0; rep < 2; rep++) {
      if (rep == 1) {
        T z = 0;
        for (int i = 0; i < 6; i++) z += gg[i];
        for (int i = 0; i < 21; i++) z += Hg[i];
        asm volatile("" :: "v"(z) : "memory");
        for (int i = 0; i < 6; i++) gg[i] = 0;
        for (int i = 0; i < 21; i++) Hg[i] = 0;
        team_sync();
      }
#endif
    for (int c = tl; c < ngc; c += L) {
      const bool wheel = c < 3;
      T jar[3], Dc = 0, Jg[3][6];
      if (wheel) {
#pragma unroll
        for (int r = 0; r < 3; r++) jar[r] = wheel_dot(W.wc[c], c, r, a) - W.wc[c].aref[r];
      } else {
        T ar[3];
        ground_get<BODY>(m, W, c - 3, Jg, ar, Dc);
#pragma unroll
        for (int r = 0; r < 3; r++) jar[r] = ground_dot(Jg, r, a) - ar[r];
      }
      if (c == tl) {
#pragma unroll
        for (int r = 0; r < 3; r++) jar0[r] = jar[r];
      }
      const T D[3] = {wheel ? W.wc[c].D[0] : Dc, wheel ? W.wc[c].D[1] : Dc, wheel ? W.wc[c].D[2] : Dc};
      const T mu = wheel ? muw : T(1), f1 = wheel ? muw : T(1), f2 = wheel ? m.fr_wheel[1] : T(1);
      const T Dm = D[0] * (wheel ? kdw : T(0.5));  // 1 / (mu^2 (1 + mu^2))
      T f[3], Cc[6];
      cone_sel(jar, mu, f1, f2, D, Dm, f, Cc);
      if (wheel) {
        T* p = wCf + 9 * c;
#pragma unroll
        for (int r = 0; r < 6; r++) p[r] = Cc[r];
#pragma unroll
        for (int r = 0; r < 3; r++) p[6 + r] = f[r];
      } else {
        T w[3][6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
          gg[i] -= Jg[0][i] * f[0] + Jg[1][i] * f[1] + Jg[2][i] * f[2];
          w[0][i] = Cc[0] * Jg[0][i] + Cc[3] * Jg[1][i] + Cc[4] * Jg[2][i];
          w[1][i] = Cc[3] * Jg[0][i] + Cc[1] * Jg[1][i] + Cc[5] * Jg[2][i];
          w[2][i] = Cc[4] * Jg[0][i] + Cc[5] * Jg[1][i] + Cc[2] * Jg[2][i];
        }
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
          for (int j = 0; j <= i; j++) Hg[i * (i + 1) / 2 + j] += Jg[0][i] * w[0][j] + Jg[1][i] * w[1][j] + Jg[2][i] * w[2][j];
      }
    }
#ifdef BB_EXP_DUP_CPASS
    }
#endif
    // base-tree contacts (full kernel), contact-parallel in world form
    // (BodyFrame): lane tl rebuilds contact b0 + tl's frame and cone force and
    // forms A = F' C F and phi = F' f; each contact's A, phi and its column
    // vectors' parameters (db, dB, hw, ball, hinge: 18 values, not the 39 of
    // J) are then broadcast over the row (DPP), and every lane adds its own
    // Hessian row sum_b w_b,row' A_b w_b,q and gradient entry -w_b,row' phi_b.
    // The row is accumulated in world vectors (base lin, Rb-frame lever sum,
    // hinge slots, ball lin, RB-frame lever sum) and turned into dof entries
    // once per iteration.
    T hb[NV], gb = 0;
#pragma unroll
    for (int i = 0; i < NV; i++) hb[i] = 0;
    if constexpr (BODY) {
#ifdef BB_EXP_DUP_FBODY  // timing experiment: the base-tree contact pass twice
     for (int rep = 0; rep < 2; rep++) {
      if (rep == 1) { T z = 0; for (int i = 0; i < NV; i++) z += hb[i]; asm volatile("" :: "v"(z), "v"(gb) : "memory");
                      for (int i = 0; i < NV; i++) hb[i] = 0; gb = 0; }
#endif
      // this row's column vector w_row = ev + [ang] rc x (db | dB) + [hinge slot] hw, times -ball on ball rows
      const bool r_ang = (row >= 3 && row < 6) || row >= 12, r_ball = row >= 9;
      const int r_h = (row >= 6 && row < 9) ? row - 6 : -2;
      const int r_e = row < 3 ? row : ((row >= 9 && row < 12) ? row - 9 : -1);
      T rc[3] = {0, 0, 0};
      if (r_ang) {
        const T* R = row < 6 ? W.P.Rb : W.P.RB;
        const int k = row < 6 ? row - 3 : row - 12;
        rc[0] = R[k]; rc[1] = R[3 + k]; rc[2] = R[6 + k];
      }
      T Ul[3] = {0, 0, 0}, Yb[3] = {0, 0, 0}, Ub[3] = {0, 0, 0}, YB[3] = {0, 0, 0}, hs[3] = {0, 0, 0};
      for (int b0 = 0; b0 < nb; b0 += L) {  // team-uniform
        T A[6] = {0, 0, 0, 0, 0, 0}, ph[3] = {0, 0, 0}, db[3] = {0, 0, 0}, dB[3] = {0, 0, 0}, hw[3] = {0, 0, 0};
        T mb = 0;  // -ball
        int hinge = -1;
        if (b0 + tl < nb) {
          T bcv[NBF];
          body_load(W, b0 + tl, bcv);
          BodyFrame<T> bf;
          body_frame(m, bcv, W.P, W.vi, bf);
          T V[3], jar[3];
          body_V(bf, W.P, a, V);
#pragma unroll
          for (int r = 0; r < 3; r++) jar[r] = dot3(bf.F[r], V) - bf.aref[r];
          const T D[3] = {bf.D, bf.D, bf.D};
          T f[3], Cc[6];
          cone_sel(jar, T(1), T(1), T(1), D, bf.D * T(0.5), f, Cc);
          // G = C F (rows r), A = F' G, phi = F' f
          T G[3][3];
#pragma unroll
          for (int i = 0; i < 3; i++) {
            G[0][i] = Cc[0] * bf.F[0][i] + Cc[3] * bf.F[1][i] + Cc[4] * bf.F[2][i];
            G[1][i] = Cc[3] * bf.F[0][i] + Cc[1] * bf.F[1][i] + Cc[5] * bf.F[2][i];
            G[2][i] = Cc[4] * bf.F[0][i] + Cc[5] * bf.F[1][i] + Cc[2] * bf.F[2][i];
            ph[i] = bf.F[0][i] * f[0] + bf.F[1][i] * f[1] + bf.F[2][i] * f[2];
          }
          auto Aij = [&](int i, int j) { return bf.F[0][i] * G[0][j] + bf.F[1][i] * G[1][j] + bf.F[2][i] * G[2][j]; };
          A[0] = Aij(0, 0); A[1] = Aij(1, 1); A[2] = Aij(2, 2); A[3] = Aij(0, 1); A[4] = Aij(0, 2); A[5] = Aij(1, 2);
#pragma unroll
          for (int i = 0; i < 3; i++) { db[i] = bf.db[i]; dB[i] = bf.dB[i]; hw[i] = bf.hw[i]; }
          mb = -bf.ball;
          hinge = bf.hinge;
        }
        const int cnt = nb - b0;
        static_for<L>([&](auto jc_) {
          constexpr int j = decltype(jc_)::value;
          if (j < cnt) {  // team-uniform
            const int hj = __builtin_amdgcn_update_dpp(0, hinge, 0x150 + j, 0xF, 0xF, false);
            T Ab[6], pb[3], dbb[3], dBb[3], hwb[3];
#pragma unroll
            for (int r = 0; r < 6; r++) Ab[r] = bcast<j>(A[r]);
#pragma unroll
            for (int r = 0; r < 3; r++) {
              pb[r] = bcast<j>(ph[r]); dbb[r] = bcast<j>(db[r]); dBb[r] = bcast<j>(dB[r]); hwb[r] = bcast<j>(hw[r]);
            }
            const T mbb = bcast<j>(mb);
            T w[3], cx[3], wx[3];
#pragma unroll
            for (int r = 0; r < 3; r++) cx[r] = row < 6 ? dbb[r] : dBb[r];
            cross3(wx, rc, cx);
#pragma unroll
            for (int r = 0; r < 3; r++) {
              T x = (r_e == r ? T(1) : T(0)) + (r_ang ? wx[r] : T(0)) + (r_h == hj ? hwb[r] : T(0));
              w[r] = r_ball ? mbb * x : x;
            }
            const T u[3] = {Ab[0] * w[0] + Ab[3] * w[1] + Ab[4] * w[2], Ab[3] * w[0] + Ab[1] * w[1] + Ab[5] * w[2],
                            Ab[4] * w[0] + Ab[5] * w[1] + Ab[2] * w[2]};
            gb -= w[0] * pb[0] + w[1] * pb[1] + w[2] * pb[2];
            T y[3], yB[3];
            cross3(y, dbb, u);
            cross3(yB, dBb, u);
#pragma unroll
            for (int r = 0; r < 3; r++) {
              Ul[r] += u[r];
              Yb[r] += y[r];
              Ub[r] += mbb * u[r];
              YB[r] += mbb * yB[r];
            }
            const T hu = hwb[0] * u[0] + hwb[1] * u[1] + hwb[2] * u[2];
#pragma unroll
            for (int r = 0; r < 3; r++) hs[r] += hj == r ? hu : T(0);
          }
        });
      }
      // dof entries: base ang k = Rb_k . Yb, ball ang k = RB_k . YB
#pragma unroll
      for (int k = 0; k < 3; k++) {
        hb[k] = Ul[k];
        hb[3 + k] = W.P.Rb[k] * Yb[0] + W.P.Rb[3 + k] * Yb[1] + W.P.Rb[6 + k] * Yb[2];
        hb[6 + k] = hs[k];
        hb[9 + k] = Ub[k];
        hb[12 + k] = W.P.RB[k] * YB[0] + W.P.RB[3 + k] * YB[1] + W.P.RB[6 + k] * YB[2];
      }
#ifdef BB_EXP_DUP_FBODY
     }
#endif
    }
    PH(0)
    // ---- (2) ball-block sums of the team-summed ground contacts (DPP)
    if (gsum) {
#ifdef BB_EXP_DUP_GSUM  // timing experiment: the 27 team sums twice
      {
        T z = 0;
#pragma unroll
        for (int i = 0; i < 6; i++) z += tsum(gg[i] * T(0.5));
#pragma unroll
        for (int i = 0; i < 21; i++) z += tsum(Hg[i] * T(0.5));
        asm volatile("" :: "v"(z) : "memory");
      }
#endif
      tsum_n(gg);  // the 27 sums interleaved: no DPP hazard waits (81 s_nop per iteration before)
      tsum_n(Hg);
    }
    team_sync();  // contact f and C visible to every row owner
    PH(1)
    // ---- (3) gradient, row i: (M a)_i - qfs_i - sum_w J_w[:,i]' f_w (+ ground)
    T h[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) h[k] = BB_HROW(k);  // dense M row
    T Ma = 0;
#pragma unroll
    for (int k = 0; k < NV; k++) Ma += h[k] * a[k];
    const T mq = rowl ? Ma - qfs_i : T(0);
    T gi = mq;
    static_for<3>([&](auto wc_) {
      constexpr int w = decltype(wc_)::value;
      const int p = wheel_pos(row, w);
      if (p >= 0) {
        const WheelCon<T>& C = W.wc[w];
        const T* q = wCf + 9 * w + 6;
        gi -= C.J[0][p] * q[0] + C.J[1][p] * q[1] + C.J[2][p] * q[2];
      }
    });
    if (gsum) {
#pragma unroll
      for (int i = 0; i < 6; i++) gi += row == 9 + i ? gg[i] : T(0);
    }
    gi = rowl ? gi + gb : T(0);
    const T gn = tsum(gi * gi);
    // MuJoCo's gradient stop (mj_solPrimal: scale * ||grad|| < tolerance after an
    // iteration; the first iteration always runs), without the sqrt
    if (it > 0 && m.scale * m.scale * gn < m.tol * m.tol) break;
    PH(2)
    // ---- (4) Hessian row: M row + wheel blocks + ground block
    // J[:, p]' C J for a contact: w = C J[:, p] (C packed xx,yy,zz,xy,xz,yz)
    auto cw = [](const T* C, T j0, T j1, T j2, T& w0, T& w1, T& w2) {
      w0 = C[0] * j0 + C[3] * j1 + C[4] * j2;
      w1 = C[3] * j0 + C[1] * j1 + C[5] * j2;
      w2 = C[4] * j0 + C[5] * j1 + C[2] * j2;
    };
#ifdef BB_EXP_DUP_HESS  // timing experiment: the wheel blocks of the Hessian row twice
    {
      T h2[NV];
#pragma unroll
      for (int k = 0; k < NV; k++) h2[k] = h[k] * T(0.5);
      static_for<3>([&](auto wc_) {
        constexpr int w = decltype(wc_)::value;
        const int p = wheel_pos(row, w);
        if (p >= 0) {
          const WheelCon<T>& C = W.wc[w];
          T w0, w1, w2;
          cw(wCf + 9 * w, C.J[0][p], C.J[1][p], C.J[2][p], w0, w1, w2);
#pragma unroll
          for (int q = 0; q < 13; q++) h2[wheel_col(q, w)] += w0 * C.J[0][q] + w1 * C.J[1][q] + w2 * C.J[2][q];
        }
      });
      T acc = 0;
#pragma unroll
      for (int k = 0; k < NV; k++) acc += h2[k];
      asm volatile("" :: "v"(acc) : "memory");
    }
#endif
    static_for<3>([&](auto wc_) {
      constexpr int w = decltype(wc_)::value;
      const int p = wheel_pos(row, w);
      if (p >= 0) {
        const WheelCon<T>& C = W.wc[w];
        T w0, w1, w2;
        cw(wCf + 9 * w, C.J[0][p], C.J[1][p], C.J[2][p], w0, w1, w2);
#pragma unroll
        for (int q = 0; q < 13; q++) h[wheel_col(q, w)] += w0 * C.J[0][q] + w1 * C.J[1][q] + w2 * C.J[2][q];
      }
    });
    if (gsum) {
#pragma unroll
      for (int ai = 0; ai < 6; ai++)
#pragma unroll
        for (int b = 0; b < 6; b++) {
          const T v = Hg[ai >= b ? ai * (ai + 1) / 2 + b : b * (b + 1) / 2 + ai];
          h[9 + b] += row == 9 + ai ? v : T(0);
        }
    }
    if constexpr (BODY) {
#pragma unroll
      for (int k = 0; k < NV; k++) h[k] += hb[k];
    }
    T hdi = 0;
#pragma unroll
    for (int k = 0; k < NV; k++) hdi = row == k ? h[k] : hdi;
    PH(3)
    // ---- (5) factorise and solve
    T diag[NV], s[NV], sown;
#ifdef BB_EXP_DUP_CHOL  // timing experiment (tools/lib_bench): the factorisation twice
    {
      T h2[NV], d2[NV];
#pragma unroll
      for (int k = 0; k < NV; k++) h2[k] = h[k];
      chol_rows(h2, hdi, d2, tl);
      asm volatile("" :: "v"(d2[NV - 1]), "v"(h2[NV - 2]) : "memory");
    }
#endif
    chol_rows(h, hdi, diag, tl);
    PH(4)
#ifdef BB_EXP_DUP_TRSV  // timing experiment: the two triangular sweeps twice
    {
      T s2[NV], so2;
      chol_solve_rows(h, diag, gi, s2, so2, tl, &W.u.hes.cj[0][0][0]);
      asm volatile("" :: "v"(s2[0]), "v"(so2) : "memory");
      team_sync();
    }
#endif
    chol_solve_rows(h, diag, gi, s, sown, tlx, &W.u.hes.cj[0][0][0]);  // cj is dead after the Hessian
    T d0 = tsum(sown * gi);
    bool fin = true;
#pragma unroll
    for (int i = 0; i < NV; i++) fin = fin && isfinite(s[i]);
    if (!fin || !(d0 < 0)) {
      // roundoff-indefinite Hessian: diagonal Newton from this row, then replicated
      sown = rowl ? -gi / maxT(W.H[hidx(row, row)], T(1e-30)) : T(0);
      static_for<NV>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        s[k] = bcast<k>(sown);
      });
      d0 = tsum(sown * gi);
      if (!(d0 < 0)) break;
    }
    PH(5)
    // ---- (6) exact line search
    T Ms = 0;
#pragma unroll
    for (int k = 0; k < NV; k++) Ms += BB_HROW(k) * s[k];
    const T sMs = tsum(sown * Ms), gs = tsum(sown * mq);
    // this lane's first contact's term from its jar; later rounds rebuild theirs
    LsTerm<T> lt;
    if (tl < ngc) {
      const bool wheel = tl < 3;
      T x[3], Dc[3];
      if (wheel) {
        const WheelCon<T>& C = W.wc[tl];
#pragma unroll
        for (int r = 0; r < 3; r++) { x[r] = wheel_dot(C, tl, r, s); Dc[r] = C.D[r]; }
      } else {
        T Jg[3][6], ar[3], D;
        ground_get<BODY>(m, W, tl - 3, Jg, ar, D);
#pragma unroll
        for (int r = 0; r < 3; r++) { x[r] = ground_dot(Jg, r, s); Dc[r] = D; }
      }
      const T mu = wheel ? muw : T(1), f1 = wheel ? muw : T(1), f2 = wheel ? m.fr_wheel[1] : T(1);
      lt.prep(jar0, x, mu, f1, f2, Dc, Dc[0] * (wheel ? kdw : T(0.5)));
    } else {
      ls_term<BODY>(m, W, tl, ng, nc, a, s, kdw, lt);  // a base-tree contact (rebuilt), or none
    }
    LineSearch<T> lsr;
    bool ls_ok = false;
#ifdef BB_EXP_DUP_LS  // timing experiment: the line search twice (first result discarded)
    auto line_search = [&](LineSearch<T>& lsr, bool& ls_ok) {
      lsr.init(d0);
      ls_ok = false;
      for (int ls = 1; ls <= m.ls_maxiter; ls++) {
        const T alpha = lsr.alpha;
        T d1p = 0, d2p = 0, dmp = 0;
        lt.eval(alpha, d1p, d2p, dmp);
        for (int c = tl + L; c < nc; c += L) {
          LsTerm<T> lc;
          ls_term<BODY>(m, W, c, ng, nc, a, s, kdw, lc);
          lc.eval(alpha, d1p, d2p, dmp);
        }
        const T d1 = gs + alpha * sMs + tsum(d1p);
        const T d2 = sMs + tsum(d2p);
        const T dmag = fabs(gs) + fabs(alpha * sMs) + tsum(dmp);
        if (fabs(d1) <= m.ls_tol * fabs(d0) || fabs(d1) <= T(32) * eps_of<T>() * dmag) { ls_ok = true; break; }
        if (!(d1 == d1)) break;
        lsr.update(d1, d2);
        const bool up = lsr.alpha > lsr.prev;
        const T big = T(1e30);
        const T kv = tmin(lsr.crosses(lt.kink) ? (up ? lt.kink : -lt.kink) : big);
        const T ks = up ? kv : -kv;
        lsr.dx = kv < big ? fabs(ks - lsr.prev) : lsr.dx;
        lsr.alpha = kv < big ? ks : lsr.alpha;
      }
    };
    {
      LineSearch<T> l2;
      bool ok2;
      line_search(l2, ok2);
      asm volatile("" :: "v"(l2.alpha), "v"(int(ok2)) : "memory");
    }
    PH(8)
    line_search(lsr, ls_ok);
#else
    lsr.init(d0);
    PH(8)
    for (int ls = 1; ls <= m.ls_maxiter; ls++) {
      const T alpha = lsr.alpha;
      T d1p = 0, d2p = 0, dmp = 0;
      lt.eval(alpha, d1p, d2p, dmp);
      for (int c = tl + L; c < nc; c += L) {
        LsTerm<T> lc;
        ls_term<BODY>(m, W, c, ng, nc, a, s, kdw, lc);
        lc.eval(alpha, d1p, d2p, dmp);
      }
      // phi' decides most evaluations: the magnitude bound (roundoff test) and
      // phi'' (the next trial) are summed only when it does not
      const T d1 = gs + alpha * sMs + tsum(d1p);
      if (fabs(d1) <= m.ls_tol * fabs(d0)) { ls_ok = true; break; }
      const T dmag = fabs(gs) + fabs(alpha * sMs) + tsum(dmp);
      if (fabs(d1) <= T(32) * eps_of<T>() * dmag) { ls_ok = true; break; }
      if (!(d1 == d1)) break;
      const T d2 = sMs + tsum(d2p);
      lsr.update(d1, d2);
      const bool up = lsr.alpha > lsr.prev;
      const T big = T(1e30);
      const T kv = tmin(lsr.crosses(lt.kink) ? (up ? lt.kink : -lt.kink) : big);
      const T ks = up ? kv : -kv;
      lsr.dx = kv < big ? fabs(ks - lsr.prev) : lsr.dx;
      lsr.alpha = kv < big ? ks : lsr.alpha;
    }
#endif
    if (!ls_ok) lsr.alpha = lsr.fallback();
    PH(9)
    const T alpha = lsr.alpha;
    if (!(alpha > 0)) break;
    // the cost change of the step (MuJoCo's improvement test below), closed form on
    // the line: alpha s'(Ma - qfs) + alpha^2 s'Ms / 2 + sum_c phi_c(alpha) - phi_c(0)
    T dc = lt.cost(alpha) - lt.cost(T(0));
    for (int c = tl + L; c < nc; c += L) {  // contacts past the team's lanes (full kernel only)
      LsTerm<T> lc;
      ls_term<BODY>(m, W, c, ng, nc, a, s, kdw, lc);
      dc += lc.cost(alpha) - lc.cost(T(0));
    }
    const T dcost = alpha * (gs + T(0.5) * alpha * sMs) + tsum(dc);
    T sn = 0, an2 = 0;
#pragma unroll
    for (int i = 0; i < NV; i++) { a[i] += alpha * s[i]; sn += s[i] * s[i]; an2 += a[i] * a[i]; }
    PH(6)
    if (alpha * alpha * sn <= T(1e-30) + m.step_rel2 * (1 + an2)) { it++; break; }
    // MuJoCo's improvement stop (mj_solPrimal: scale * (oldcost - cost) < tolerance)
    if (-m.scale * dcost < m.tol) { it++; break; }
  }
  PH(7)
#undef BB_HROW
  if constexpr (BODY) {
    PH_FLUSH_BODY((Team{L, tl}))
  } else {
    PH_FLUSH((Team{L, tl}))
  }
  return it;
}

// collide_ground (bb_physics.h) spread over the team: the prisms under the
// ball's AABB are enumerated in MuJoCo's order (row-major over the sub-grid,
// two triangles per cell in sliding-window order), 16 per round, one per
// lane; hits are compacted in that order with a ballot, so the contact list
// (and the MAXG cap) is exactly the serial one.
template <typename T>
__device__ __forceinline__ int collide_team(const ModelT<T>& m, const Kin<T>& k, const T* v, const float* hf,
                                            T size_z, T* g, int* overflow, int tl) {
  const T r = m.ball_r;
  const T* c = k.c;
  const T sx = m.hf_sx, sy = m.hf_sy, zb = m.hf_bottom;
  const T xmin = c[0] - r, xmax = c[0] + r, ymin = c[1] - r, ymax = c[1] + r, zmin = c[2] - r, zmax = c[2] + r;
  // negated form: a NaN ball position (diverged stage state) forms no cell index
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
  const int ncol = cmax - cmin + 1;
  const int np = 2 * ncol - 2;            // prisms per grid row
  const int total = (rmax - rmin) * (np > 0 ? np : 0);
  const T dx = 2 * sx / N1, dy = 2 * sy / N1;
  (void)v;
  const int team_shift = team_shift_of(L);
  int ng = 0;
  // the heights of prism P's three top vertices; the next round's are loaded while this round
  // is tested, so a round does not wait for its loads (one wave per SIMD hides no latency)
  auto heights = [&](int P, float (&h)[3]) {
    if (P < total) {
      const int rr = rmin + P / np, p = P % np;
#pragma unroll
      for (int t = 0; t < 3; t++) {
        const int vt = p + t;
        h[t] = hf[(rr + (vt & 1)) * HF_N + cmin + (vt >> 1)];
      }
    }
  };
  float hnext[3] = {0.f, 0.f, 0.f};
  heights(tl, hnext);
  for (int base = 0; base < total; base += L) {
    const int P = base + tl;
    bool hit = false;
    T nn[3] = {0, 0, 1}, dist = 0;
    const float hcur[3] = {hnext[0], hnext[1], hnext[2]};
    heights(P + L, hnext);
    if (P < total) {
      const int rr = rmin + P / np, p = P % np;
      T V[3][3];
#pragma unroll
      for (int t = 0; t < 3; t++) {
        const int vt = p + t, cc = cmin + (vt >> 1), ri = rr + (vt & 1);
        V[t][0] = dx * cc - sx;
        V[t][1] = dy * ri - sy;
        V[t][2] = T(hcur[t]) * size_z;
        (void)ri; (void)cc;
      }
      if (!(V[0][2] < zmin && V[1][2] < zmin && V[2][2] < zmin)) {
        const T bx0 = minT(V[0][0], minT(V[1][0], V[2][0])), bx1 = maxT(V[0][0], maxT(V[1][0], V[2][0]));
        const T by0 = minT(V[0][1], minT(V[1][1], V[2][1])), by1 = maxT(V[0][1], maxT(V[1][1], V[2][1]));
        const T ztop = maxT(V[0][2], maxT(V[1][2], V[2][2]));
        const T ex = maxT(T(0), maxT(bx0 - c[0], c[0] - bx1));
        const T ey = maxT(T(0), maxT(by0 - c[1], c[1] - by1));
        const T ez = maxT(T(0), c[2] - ztop);
        if (ex * ex + ey * ey + ez * ez <= r * r) hit = sphere_prism(c, r, V, -zb, nn, &dist);
      }
    }
    const unsigned long long bal = __ballot(hit);
    const unsigned bits = unsigned(bal >> team_shift) & 0xFFFFu;
    const int slot = ng + __popc(bits & ((1u << tl) - 1u));
    if (hit) {
      if (slot < MAXG) {
        T* gs = g + slot * NGF;
#pragma unroll
        for (int i = 0; i < 3; i++) gs[GF_N + i] = nn[i];
        gs[GF_DIST] = dist;
      }
    }
    ng += __popc(bits);
  }
  if (ng > MAXG) { ng = MAXG; *overflow = 1; }  // ng counts every hit: team-uniform
  return ng;
}

// store one base-tree contact (slot already compacted)
template <typename T>
__device__ __forceinline__ void put_body(T* bc, T* spill, int slot, const T* n, const T* pos, T dist, int b1, int b2) {
  T* s = body_slot(bc, spill, slot);
#pragma unroll
  for (int i = 0; i < 3; i++) { s[BF_N + i] = n[i]; s[BF_P + i] = pos[i]; }
  s[BF_DIST] = dist;
  s[BF_CODE] = T(8 * b1 + b2);
}

// Conservative prune before the exact prism test: every point of a capsule or
// cylinder g lies within g.r, coordinate-wise, of its axis segment c + t a,
// |t| <= hh.  It can only reach the prism (xy in its top triangle, z below the
// highest top vertex) if some segment point has x, y within g.r of the
// triangle's bounding box and z - g.r below that top.  False only when no
// contact is possible, so the exact SAT keeps deciding every contact.  The
// slab reciprocals are per geom (Reach), not per prism.
template <typename T>
struct Reach {
  T c[3], a[3], hh, r, ia[2];
  bool par[2];  // axis parallel to the slab's planes
};

template <typename T>
__device__ __forceinline__ void make_reach(const Seg<T>& g, Reach<T>& R) {
#pragma unroll
  for (int i = 0; i < 3; i++) { R.c[i] = g.c[i]; R.a[i] = g.a[i]; }
  R.hh = g.hh; R.r = g.r;
#pragma unroll
  for (int ax = 0; ax < 2; ax++) {
    R.par[ax] = fabs(g.a[ax]) < T(1e-12);
    R.ia[ax] = R.par[ax] ? T(0) : T(1) / g.a[ax];
  }
}

template <typename T>
__device__ __forceinline__ bool prism_may_hit(const Reach<T>& g, const T (&V)[3][3]) {
  T t0 = -g.hh, t1 = g.hh;
  bool out = false;
#pragma unroll
  for (int ax = 0; ax < 2; ax++) {
    const T lo = minT(V[0][ax], minT(V[1][ax], V[2][ax])) - g.r;
    const T hi = maxT(V[0][ax], maxT(V[1][ax], V[2][ax])) + g.r;
    if (g.par[ax]) {
      out = out || g.c[ax] < lo || g.c[ax] > hi;
    } else {
      const T ta = (lo - g.c[ax]) * g.ia[ax], tb = (hi - g.c[ax]) * g.ia[ax];
      t0 = maxT(t0, minT(ta, tb));
      t1 = minT(t1, maxT(ta, tb));
    }
  }
  if (out || t0 > t1) return false;
  const T ztop = maxT(V[0][2], maxT(V[1][2], V[2][2]));
  const T zmin = g.c[2] + minT(t0 * g.a[2], t1 * g.a[2]) - g.r;
  return zmin <= ztop;
}

// Fast-path test: can any base-tree contact exist at this configuration?
// Exact for ball x {tower, sticks}; for hfield x geom it asks whether any
// heightfield vertex under the geom's AABB reaches the geom's lowest point --
// MuJoCo's own prism pre-filter (a prism whose three top vertices are below
// the geom's AABB is skipped), so "no" is exact and "yes" sends the env to the
// full kernel.  Team-uniform result.
template <typename T>
__device__ bool body_candidates(const ModelT<T>& m, const Kin<T>& k, const float* hf, T size_z, T hz, int tl) {
  bool cand = false;
  // lane gi < 6 places geom gi once (lanes 0..2 also test it against the
  // ball) and screens it against the terrain: its AABB must reach the
  // terrain's top (hz) and overlap the grid.  Only the geoms that pass are
  // walked, by the whole team -- rather than every lane placing all six.
  bool reach = false;
  if (tl < 6) {
    Seg<T> g;
    body_geom(m, k, tl, g);
    if (tl < 3) {
      T dist, n[3], pos[3];
      cand = tl == 0 ? sphere_cylinder(k.c, m.ball_r, g, dist, n, pos) : sphere_capsule(k.c, m.ball_r, g, dist, n, pos);
    }
    if (hf) {
      const T sx = m.hf_sx, sy = m.hf_sy, zb = m.hf_bottom;
      T lo[3], hi[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        const T ai = fabs(g.a[i]);
        const T rad = T(1) - ai * ai;
        const T ext = tl == 0 ? g.hh * ai + g.r * sqrt(rad > 0 ? rad : T(0)) : g.hh * ai + g.r;
        lo[i] = g.c[i] - ext; hi[i] = g.c[i] + ext;
      }
      // negated: a NaN pose skips the geom (no cell index from it)
      reach = lo[2] <= hz && lo[0] <= sx && hi[0] >= -sx && lo[1] <= sy && hi[1] >= -sy && lo[2] <= size_z &&
              hi[2] >= -zb;
    }
  }
  unsigned todo = unsigned(__ballot(reach) >> team_shift_of(L)) & 0x3Fu;  // team-uniform
  if (hf) {
    const T sx = m.hf_sx, sy = m.hf_sy;
    const int N1 = HF_N - 1;
    while (todo) {
      const int gi = __builtin_ctz(todo);
      todo &= todo - 1;
      Seg<T> g;
      body_geom(m, k, gi, g);
      Reach<T> gr;
      make_reach(g, gr);
      T lo[3], hi[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        const T ai = fabs(g.a[i]);
        const T rad = T(1) - ai * ai;
        const T ext = gi == 0 ? g.hh * ai + g.r * sqrt(rad > 0 ? rad : T(0)) : g.hh * ai + g.r;
        lo[i] = g.c[i] - ext; hi[i] = g.c[i] + ext;
      }
      int cmin = (int)floor((lo[0] + sx) / (2 * sx) * N1), cmax = (int)ceil((hi[0] + sx) / (2 * sx) * N1);
      int rmin = (int)floor((lo[1] + sy) / (2 * sy) * N1), rmax = (int)ceil((hi[1] + sy) / (2 * sy) * N1);
      cmin = cmin < 0 ? 0 : cmin; cmax = cmax > N1 ? N1 : cmax;
      rmin = rmin < 0 ? 0 : rmin; rmax = rmax > N1 ? N1 : rmax;
      if (rmax <= rmin || cmax <= cmin) continue;  // no prism
      // the full kernel's prisms (cells [rmin, rmax) x [cmin, cmax), two
      // triangles each) under its own two prunes: a candidate iff the exact
      // prism test would run on at least one of them
      const T dx = 2 * sx / N1, dy = 2 * sy / N1;
      const int nc = cmax - cmin, total = (rmax - rmin) * nc;
      for (int i = tl; i < total && !cand; i += L) {
        const int ri = rmin + i / nc, ci = cmin + i % nc;
        const T x0 = dx * ci - sx, x1 = dx * (ci + 1) - sx, y0 = dy * ri - sy, y1 = dy * (ri + 1) - sy;
        const T z00 = T(hf[ri * HF_N + ci]) * size_z, z10 = T(hf[(ri + 1) * HF_N + ci]) * size_z;
        const T z01 = T(hf[ri * HF_N + ci + 1]) * size_z, z11 = T(hf[(ri + 1) * HF_N + ci + 1]) * size_z;
        const T A[3][3] = {{x0, y0, z00}, {x0, y1, z10}, {x1, y0, z01}};
        const T B[3][3] = {{x0, y1, z10}, {x1, y0, z01}, {x1, y1, z11}};
        const bool ta = !(z00 < lo[2] && z10 < lo[2] && z01 < lo[2]) && prism_may_hit(gr, A);
        const bool tb = !(z10 < lo[2] && z01 < lo[2] && z11 < lo[2]) && prism_may_hit(gr, B);
        cand = ta || tb;
      }
    }
  }
  const unsigned bits = unsigned(__ballot(cand) >> team_shift_of(L)) & 0xFFFFu;
  return bits != 0;
}

// per-team SAT candidate list capacity (ints, in the team's W.H: free until
// mass_dense_team; 91 floats at fp32)
constexpr int CAND_CAP = 80;

// Dynamic pairs of the base-tree geoms (bb_bodycon.h), team-parallel, in the
// oracle's order: ball x {tower, stick0, stick1}, then hfield x {tower,
// stick0, stick1, wheel0..2} prism by prism.  hz: the terrain's top height
// (max(hfield) * size_z): geoms above it skip the prism loop.  Each hfield
// pair keeps its first MAXPAIR contacts in prism order (MuJoCo's
// mjMAXCONPAIR; *overflow |= 2 when a pair had more).  Contacts go to bc (the
// first MAXB_LDS, LDS) and spill (the rest, HBM).  Returns the contact count
// (team-uniform).  cand: the team's candidate list (CAND_CAP ints of LDS).

template <typename T>
__device__ int collide_body_team(const ModelT<T>& m, const Kin<T>& k, const float* hf, T size_z, T hz, T* bc,
                                 T* spill, int* overflow, int tl, int* cand) {
  const int team_shift = team_shift_of(L);
  const unsigned below = (1u << tl) - 1u;
  int nb = 0;
  auto compact = [&](bool hit) -> int {  // -> this lane's slot (valid if hit)
    const unsigned bits = unsigned(__ballot(hit) >> team_shift) & 0xFFFFu;
    const int slot = nb + __popc(bits & below);
    nb += int(__popc(bits));
    return slot;
  };
  // ball (geom1, sphere) x tower (cylinder) / sticks (capsules): lanes 0..2
  {
    bool hit = false;
    T dist = 0, n[3] = {0, 0, 1}, pos[3] = {0, 0, 0};
    if (tl < 3) {
      Seg<T> g;
      body_geom(m, k, tl, g);
      hit = tl == 0 ? sphere_cylinder(k.c, m.ball_r, g, dist, n, pos) : sphere_capsule(k.c, m.ball_r, g, dist, n, pos);
    }
    const int slot = compact(hit);
    if (hit) put_body(bc, spill, slot, n, pos, dist, 7, tl + 1);
  }
  // hfield (geom1) x convex geom, in two passes so the exact test runs on full
  // rounds.  Pass 1 walks the prisms under each geom's AABB 16 at a time with
  // the cheap conservative prunes and appends survivors, in (geom, row-major
  // prism) order, to a per-team candidate list in LDS; pass 2 runs the exact
  // body-prism SAT 16 candidates per round.  Perlin: ~230 prisms over 6 geoms
  // leave ~8 candidates per forward -- one SAT round instead of up to 8.
  // Contact order is unchanged (both passes keep list order).
  if (hf) {
    const T sx = m.hf_sx, sy = m.hf_sy, zb = m.hf_bottom;
    const int N1 = HF_N - 1;
    const T dx = 2 * sx / N1, dy = 2 * sy / N1;
    int nc = 0;  // candidates pending in cand[]
    int pair_n[6] = {0, 0, 0, 0, 0, 0};  // contacts so far per hfield pair (team-uniform)
    auto vertices = [&](int rr, int p, T (&V)[3][3]) {
#pragma unroll
      for (int t = 0; t < 3; t++) {
        const int vt = p + t, cc = (vt >> 1), ri = rr + (vt & 1);
        V[t][0] = dx * cc - sx;
        V[t][1] = dy * ri - sy;
        V[t][2] = T(hf[ri * HF_N + cc]) * size_z;
      }
    };
    auto flush = [&]() {
      team_sync();  // cand[] writes visible to the team
      for (int base = 0; base < nc; base += L) {
        bool hit = false;
        T dist = 0, n[3] = {0, 0, 1}, pos[3] = {0, 0, 0};
        int b2 = 0;
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
        int sat_path = -1;
        const unsigned long long sat_c0 = clock64();
#endif
        if (base + tl < nc) {
          const int code = cand[base + tl];
          const int gi = code >> 26, rr = (code >> 13) & 0x1FFF, p = code & 0x1FFF;
          Seg<T> g;
          body_geom(m, k, gi, g);
          T V[3][3];
          vertices(rr, p, V);
          PrismG<T> Pr;
          prism_build(Pr, V, -zb);
#ifdef BB_EXP_DUP_SAT  // timing experiment: the exact prism tests twice
          {
            T d2 = 0, n2[3], p2[3];
            const bool h2 = gi == 0 ? cylinder_prism(g, Pr, d2, n2, p2) : capsule_prism(g, Pr, d2, n2, p2);
            asm volatile("" :: "v"(d2), "v"(n2[0]), "v"(p2[0]), "v"(int(h2)) : "memory");
          }
#endif
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
          sat_path = gi == 0 ? 3 : capsule_prism_path(g, Pr);
#endif
#ifdef BB_EXP_DUP_CYL  // timing experiment: the tower's cylinder SAT once more, as a call (an inlined copy
                       // spills the pair's registers and measures the spills)
          if (gi == 0) {
            const T d2 = cylinder_prism_dup_call(g.c[0], g.c[1], g.c[2], g.a[0], g.a[1], g.a[2], g.hh, g.r, V[0][0],
                                                 V[0][1], V[0][2], V[1][0], V[1][1], V[1][2], V[2][0], V[2][1],
                                                 V[2][2], -zb);
            asm volatile("" :: "v"(d2) : "memory");
          }
#endif
          hit = gi == 0 ? cylinder_prism(g, Pr, dist, n, pos) : capsule_prism(g, Pr, dist, n, pos);
          b2 = gi + 1;  // body ids: tower 1, sticks 2-3, wheels 4-6
        }
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
        {  // SAT rounds: lanes per path, and the rounds each path ran in (the wave runs every path any lane takes)
          const int sh = team_shift_of(L);
          auto lanes = [&](bool c) { return __popc(unsigned(__ballot(c) >> sh) & 0xFFFFu); };
          const int nl = lanes(sat_path >= 0), ncy = lanes(sat_path == 3), neo = lanes(sat_path == 0),
                    nin = lanes(sat_path == 1), nap = lanes(sat_path == 2), nah = lanes(sat_path == 2 && hit);
          if (tl == 0) {
            atomicAdd(&bb_phase_cycles[90], 1ull);
            atomicAdd(&bb_phase_cycles[91], (unsigned long long)nl);
            atomicAdd(&bb_phase_cycles[92], (unsigned long long)ncy);
            atomicAdd(&bb_phase_cycles[93], (unsigned long long)neo);
            atomicAdd(&bb_phase_cycles[94], (unsigned long long)nin);
            atomicAdd(&bb_phase_cycles[95], (unsigned long long)nap);
            atomicAdd(&bb_phase_cycles[96], (unsigned long long)nah);
            atomicAdd(&bb_phase_cycles[97], (unsigned long long)(nap > 0));
            atomicAdd(&bb_phase_cycles[98], (unsigned long long)(nin + ncy > 0));
            atomicAdd(&bb_phase_cycles[99], clock64() - sat_c0);
          }
        }
#endif
        // per-pair cap: a hit is kept while its pair has fewer than MAXPAIR
        // (candidates of one pair sit in consecutive lanes, in prism order)
        bool keep = hit;
#pragma unroll
        for (int g = 0; g < 6; g++) {
          const unsigned gb = unsigned(__ballot(hit && b2 == g + 1) >> team_shift) & 0xFFFFu;
          if (hit && b2 == g + 1) keep = pair_n[g] + __popc(gb & below) < MAXPAIR;
          if (pair_n[g] + __popc(gb) > MAXPAIR) *overflow |= 2;
          pair_n[g] = minT(pair_n[g] + int(__popc(gb)), MAXPAIR);
        }
        const int slot = compact(keep);
        if (keep) put_body(bc, spill, slot, n, pos, dist, 0, b2);
      }
      team_sync();  // cand[] reads done before it is refilled
      nc = 0;
    };
    for (int gi = 0; gi < 6; gi++) {
      Seg<T> g;
      body_geom(m, k, gi, g);
      Reach<T> gr;
      make_reach(g, gr);
      const bool cyl = gi == 0;
      T lo[3], hi[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        const T ai = fabs(g.a[i]);
        const T rad = T(1) - ai * ai;
        const T ext = cyl ? g.hh * ai + g.r * sqrt(rad > 0 ? rad : T(0)) : g.hh * ai + g.r;
        lo[i] = g.c[i] - ext; hi[i] = g.c[i] + ext;
      }
      if (!(lo[2] <= hz)) continue;  // above every vertex of the terrain (or a NaN pose)
      if (!(lo[0] <= sx && hi[0] >= -sx && lo[1] <= sy && hi[1] >= -sy && lo[2] <= size_z && hi[2] >= -zb)) continue;
      int cmin = (int)floor((lo[0] + sx) / (2 * sx) * N1), cmax = (int)ceil((hi[0] + sx) / (2 * sx) * N1);
      int rmin = (int)floor((lo[1] + sy) / (2 * sy) * N1), rmax = (int)ceil((hi[1] + sy) / (2 * sy) * N1);
      cmin = cmin < 0 ? 0 : cmin; cmax = cmax > N1 ? N1 : cmax;
      rmin = rmin < 0 ? 0 : rmin; rmax = rmax > N1 ? N1 : rmax;
      const int np = 2 * (cmax - cmin + 1) - 2;
      const int total = (rmax - rmin) * (np > 0 ? np : 0);
#ifdef BB_EXP_DUP_PRUNE  // timing experiment: the prune walk twice (first pass discarded)
      for (int base = 0; base < total; base += L) {
        const int P = base + tl;
        bool ch = false;
        if (P < total) {
          const int rr = rmin + P / np, p = 2 * cmin + P % np;
          T V[3][3];
          vertices(rr, p, V);
          ch = !(V[0][2] < lo[2] && V[1][2] < lo[2] && V[2][2] < lo[2]) && prism_may_hit(gr, V);
        }
        const unsigned long long bal = __ballot(ch);
        asm volatile("" :: "s"(bal) : "memory");
      }
#endif
      // the next round's vertex heights are loaded while this round is tested (as collide_team)
      auto heights = [&](int P, float (&h)[3]) {
        if (P < total) {
          const int rr = rmin + P / np, p = 2 * cmin + P % np;
#pragma unroll
          for (int t = 0; t < 3; t++) {
            const int vt = p + t;
            h[t] = hf[(rr + (vt & 1)) * HF_N + (vt >> 1)];
          }
        }
      };
      float hnext[3] = {0.f, 0.f, 0.f};
      heights(tl, hnext);
      for (int base = 0; base < total; base += L) {
        const int P = base + tl;
        bool cand_hit = false;
        int code = 0;
        const float hcur[3] = {hnext[0], hnext[1], hnext[2]};
        heights(P + L, hnext);
        if (P < total) {
          const int rr = rmin + P / np, p = 2 * cmin + P % np;
          T V[3][3];
#pragma unroll
          for (int t = 0; t < 3; t++) {  // vertices(rr, p, V), with the prefetched heights
            const int vt = p + t;
            V[t][0] = dx * (vt >> 1) - sx;
            V[t][1] = dy * (rr + (vt & 1)) - sy;
            V[t][2] = T(hcur[t]) * size_z;
          }
          cand_hit = !(V[0][2] < lo[2] && V[1][2] < lo[2] && V[2][2] < lo[2]) && prism_may_hit(gr, V);
          code = (gi << 26) | (rr << 13) | p;
        }
        const unsigned long long bal = __ballot(cand_hit);
        const unsigned bits = unsigned(bal >> team_shift) & 0xFFFFu;
        if (cand_hit) cand[nc + __popc(bits & ((1u << tl) - 1u))] = code;
        nc += int(__popc(bits));
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
        if (tl == 0) atomicAdd(&bb_phase_cycles[19], (unsigned long long)__popc(bits));  // SAT runs
#endif
        if (nc > CAND_CAP - L) flush();
      }
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
      if (tl == 0) {  // geoms reaching the prism loop, prisms, rounds
        atomicAdd(&bb_phase_cycles[16], 1ull);
        atomicAdd(&bb_phase_cycles[17], (unsigned long long)total);
        atomicAdd(&bb_phase_cycles[18], (unsigned long long)((total + L - 1) / L));
      }
#endif
    }
    if (nc > 0) flush();
  }
  return nb;
}

// dense mass matrix (packed lower) into W.H, entry-parallel; once per forward
template <typename T>
__device__ __forceinline__ void mass_dense_team(EnvWork<T>& W, int tl) {
  for (int e = tl; e < NH; e += L) {
    int i, j;
    tri_unpack(e, i, j);
    W.H[e] = mass_entry(W.M, i, j);
  }
}

}  // namespace t16
#endif
}  // namespace bb
