// bb_step.h -- one env step = one BBotSimulation.step (ballbot_env.py:854-1036):
//   action -> ctrl (:903-907), mj_step with RK4 (:912), _get_obs (:771-811),
//   DirectionalReward + action penalty + survival bonus (:929-937, :1019),
//   termination (:982-1017).  Per env team of lanes, templated on T (see bb_physics.h).
#pragma once

#include "bb_team16.h"

namespace bb {

// Env configuration (BBotSimulation.__init__, ballbot_env.py:221-231).
struct EnvCfg {
  int max_ep_steps;        // 4000
  float max_allowed_tilt;  // 20 deg
  float max_wheel_velocity;  // 10
  float reward_scale;      // 0.01
  float action_reg_coef;   // -1e-4
  float survival_bonus;    // 0.02
  float target[2];         // DirectionalReward target_direction
  int reward_kind;         // 0 directional, 1 distance (needs pos2d; raises in ref), 2 none (host plugin)
  float goal[2], goal_scale;
};

// mj_forward for this model: returns qacc in acc (acc holds the warm start on
// entry).  Executed by a team of tm.L lanes; the per-wheel pre-phase work (frames,
// mass terms, RNE forces, contacts) runs one wheel per lane, the rest of the pre-phase (kinematics, mass,
// bias, collision) is computed redundantly by every lane of the team, the
// constraint solve is team-parallel (bb_solve.h).
template <typename T, bool BODY = true>
BB_HD int forward(const ModelT<T>& m, const T* q, const T* v, const T* ctrl, T* acc, const TerrainRef<T>& tr,
                  EnvWork<T>& W, StageOut<T>* so, const Team& tm) {
  team_sync();  // previous users of the workspace are done
  if (v != W.vi) {  // the constraint rebuilds in the solve read the velocity from the workspace
#pragma unroll
    for (int i = 0; i < NV; i++) W.vi[i] = v[i];
    team_sync();
  }
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long f_t0 = clock64();
#endif
  Kin<T>& k = W.u.pre.k;
#ifdef __HIP_DEVICE_COMPILE__
  // base/ball frames on every lane, wheel w's frame on lane w
  kinematics_base(m, q, k);
  if (tm.tl < 3) kinematics_wheel(m, q, tm.tl, k);
  team_sync();
#else
  kinematics(m, q, k);
#endif
  Mass<T>& M = W.M;
#ifdef __HIP_DEVICE_COMPILE__
  {
    // lane w: wheel w's mass terms, RNE force and contact; W.H (free until
    // mass_dense_team) holds the per-wheel terms that every lane then sums
    // in wheel order
    T (*mrw)[3] = reinterpret_cast<T (*)[3]>(W.H);
    T (*IOw)[6] = reinterpret_cast<T (*)[6]>(W.H + 9);
    T (*fw)[6] = reinterpret_cast<T (*)[6]>(W.H + 27);
    static_assert(NH >= 45, "per-wheel terms do not fit W.H");
    if (tm.tl < 3) {
      const int w = tm.tl;
      mass_wheel(m, k, w, M, W.u.pre.Iw[w], mrw[w], IOw[w]);
      T w0[3], vl[3], a0[3];
      bias_base_motion(m, k, v, w0, vl, a0);
      const T qb = -bias_wheel(m, k, W.u.pre.Iw[w], v, w, w0, vl, a0, fw[w], fw[w] + 3);
      const T cw = w == 0 ? ctrl[0] : (w == 1 ? ctrl[1] : ctrl[2]);  // no dynamic index into registers
      W.qfs[6 + w] = qb + (-m.damping * v[6 + w] + cw);
      wheel_contact(m, k, v, w, W.wc[w]);  // read after the solve's team_sync
    }
    team_sync();
    mass_finish(m, k, M, mrw, IOw);
    // qfrc_smooth = -bias + passive + actuation, straight to the workspace
    T qfs[NV];
    bias_finish(m, k, v, fw, qfs);
#pragma unroll
    for (int i = 0; i < NV; i++)
      if (i < 6 || i > 8) W.qfs[i] = -qfs[i];
    team_sync();  // W.H free again (candidate list of the body collision)
  }
#else
  build_mass(m, k, M, W.u.pre.Iw);
  {
    // qfrc_smooth = -bias + passive + actuation, straight to the workspace
    T qfs[NV];
    bias_forces(m, k, W.u.pre.Iw, v, qfs);
#pragma unroll
    for (int i = 0; i < NV; i++) qfs[i] = -qfs[i];
#pragma unroll
    for (int w = 0; w < 3; w++) qfs[6 + w] += -m.damping * v[6 + w] + ctrl[w];
#pragma unroll
    for (int i = 0; i < NV; i++) W.qfs[i] = qfs[i];
  }
#pragma unroll
  for (int w = 0; w < 3; w++) wheel_contact(m, k, v, w, W.wc[w]);
#endif
  const GStore<T> st{W.g, 1};
  int overflow = 0;
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long f_t1 = clock64();
#endif
#ifdef __HIP_DEVICE_COMPILE__
  const int ng = tr.hf ? t16::collide_team(m, k, v, tr.hf, tr.size_z, W.g, &overflow, tm.tl) : 0;
  int nb = 0;
  if constexpr (BODY) {
#if defined(BB_PHASE_CLOCKS)
    const unsigned long long b_t0 = clock64();
#endif
    // W.H is free until mass_dense_team below: it holds the SAT candidate list
    static_assert(sizeof(W.H) >= t16::CAND_CAP * sizeof(int), "candidate list does not fit W.H");
#ifdef BB_EXP_DUP_BODYCOL  // timing experiment (tools/lib_bench): the base-tree collision twice
    { int ov2 = 0; (void)t16::collide_body_team(m, k, tr.hf, tr.size_z, tr.hz, W.bc, W.bspill, &ov2, tm.tl,
                                                 reinterpret_cast<int*>(W.H)); }
    asm volatile("" ::: "memory");
#endif
    nb = t16::collide_body_team(m, k, tr.hf, tr.size_z, tr.hz, W.bc, W.bspill, &overflow, tm.tl,
                                reinterpret_cast<int*>(W.H));
#if defined(BB_PHASE_CLOCKS)
    if (tm.tl == 0) {  // full kernel: forwards, body contacts, body-collision cycles
      atomicAdd(&bb_phase_cycles[12], 1ull);
      atomicAdd(&bb_phase_cycles[13], (unsigned long long)nb);
      atomicAdd(&bb_phase_cycles[14], clock64() - b_t0);
      W.dbg_nb += nb;
    }
#endif
  } else {
    // fast path: no base-tree contact support compiled in; configurations that
    // could have one abort here and are re-run by the full kernel
    if (t16::body_candidates(m, k, tr.hf, tr.size_z, tr.hz, tm.tl)) return -1;
  }
#else
  const int ng = tr.hf ? collide_ground(m, k, v, tr.hf, tr.size_z, st, &overflow) : 0;
#endif
#if defined(BB_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
  if (tm.tl == 0) {
    const unsigned long long f_t2 = clock64();
    atomicAdd(&bb_phase_cycles[8], f_t1 - f_t0);
    atomicAdd(&bb_phase_cycles[9], f_t2 - f_t1);
    atomicAdd(&bb_phase_cycles[10], 1ull);
  }
#endif
#pragma unroll
  for (int i = 0; i < 9; i++) { W.P.Rb[i] = k.Rb[i]; W.P.RB[i] = k.RB[i]; }  // Jacobian rebuilds in the solve
#pragma unroll
  for (int i = 0; i < 3; i++) { W.P.pb[i] = k.pb[i]; W.P.pB[i] = k.pB[i]; }
  if (so) {
    T qb[4] = {q[3], q[4], q[5], q[6]};
    qnormalize(qb);
    so->quat_b[0] = qb[0]; so->quat_b[1] = qb[1]; so->quat_b[2] = qb[2]; so->quat_b[3] = qb[3];
    mv3(so->w_world, k.Rb, v + 3);
    // subtree_com[base] - xpos[base] = Rb * mr / mt
    T cl[3] = {M.mr[0] / M.mt, M.mr[1] / M.mt, M.mr[2] / M.mt}, cw[3], t[3];
    mv3(cw, k.Rb, cl);
    cross3(t, so->w_world, cw);
    so->v_com[0] = v[0] + t[0]; so->v_com[1] = v[1] + t[1]; so->v_com[2] = v[2] + t[2];
    so->pb[0] = q[0]; so->pb[1] = q[1]; so->pb[2] = q[2];
    so->ng = ng; so->overflow = overflow;
#ifdef __HIP_DEVICE_COMPILE__
    so->nb = nb;
#else
    so->nb = 0;
#endif
  }
  bool ok = true;
#pragma unroll
  for (int i = 0; i < NV; i++) ok = ok && isfinite(acc[i]);
  if (!ok) {
#pragma unroll
    for (int i = 0; i < NV; i++) acc[i] = 0;
  }
#ifdef __HIP_DEVICE_COMPILE__
  // 16-lane DPP-row solve: smooth force and dense M staged in the team's LDS
  t16::mass_dense_team(W, tm.tl);
  team_sync();
  if constexpr (!BODY) t16::ground_setup(m, W, ng, tm.tl);  // into the mass blocks: after mass_dense_team

#if defined(BB_PHASE_CLOCKS)
  const unsigned long long s_t0 = clock64();
#endif
#ifdef BB_EXP_DUP_SOLVE_FULL  // timing experiment: the full kernel's constraint solve twice
  if constexpr (BODY) {
    T acc2[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) acc2[i] = acc[i];
    (void)t16::solve16<BODY>(m, W, ng, nb, acc2, tm.tl);
    asm volatile("" ::: "memory");
    team_sync();
  }
#endif
  const int it = t16::solve16<BODY>(m, W, ng, nb, acc, tm.tl);
#if defined(BB_PHASE_CLOCKS)
  if (BODY && tm.tl == 0) {  // full-kernel solve cycles and Newton iterations
    atomicAdd(&bb_phase_cycles[15], clock64() - s_t0);
    atomicAdd(&bb_phase_cycles[20], (unsigned long long)it);
  }
  if (tm.tl == 0) {  // Newton iterations per forward: max, histogram in buckets of 2
    atomicMax(&bb_phase_cycles[21], (unsigned long long)it);
    atomicAdd(&bb_phase_cycles[22 + (it / 2 < 9 ? it / 2 : 9)], 1ull);
  }
#endif
#else
  const int it = solve_team(m, W, W.qfs, ng, acc, tm);
#endif
  if (so) so->iters = it;
  return it;
}

template <typename T>
BB_HD bool vec_bad(const T* x, int n) {  // MuJoCo's mju_isBad over x[0..n): NaN or |x| > mjMAXVAL = 1e10
  bool bad = false;
#pragma unroll
  for (int i = 0; i < n; i++) bad = bad || !(fabs(x[i]) <= T(1e10));
  return bad;
}

// mj_step with integrator RK4 = mj_forward + mj_checkAcc + mj_RungeKutta(N=4) + mj_advance.
// warm: qacc_warmstart (each stage's constraint solve saves its qacc).
// mj_checkAcc: a bad qacc after the first forward resets the data (qpos0, zero
// velocity, warm start and ctrl; no height offset) and repeats that forward;
// *acc_reset reports it.  ctrl is zeroed then, as mj_resetData zeroes d->ctrl.
template <typename T, bool BODY = true>
BB_HD int rk4_step(const ModelT<T>& m, T* q, T* v, T* warm, T* ctrl, const TerrainRef<T>& tr,
                   EnvWork<T>& W, StageOut<T>& so, const Team& tm, bool* acc_reset) {
  const T h = m.h;
  // the RK context lives in the workspace (written identically by every
  // lane of the team); only the stage state and the warm start are in registers
  T* q0 = W.q0;
  T* v0 = W.v0;
  T* vs = W.vs;
  T* as = W.as;
  team_sync();
#pragma unroll
  for (int i = 0; i < NQ; i++) q0[i] = q[i];
#pragma unroll
  for (int i = 0; i < NV; i++) v0[i] = v[i];
  int iters = 0;
#pragma unroll 1
  for (int stage = 0; stage < 4; stage++) {
    const T a = stage == 3 ? T(1) : T(0.5);  // RK4 Butcher A (sub-diagonal)
    {
      // stage state X0 (+) h a (v_prev, a_prev), kept in the workspace so that
      // nothing but the warm start stays in registers across the solve
      T qi[NQ], vi[NV];
#pragma unroll
      for (int i = 0; i < NQ; i++) qi[i] = q0[i];
      if (stage == 0) {
#pragma unroll
        for (int i = 0; i < NV; i++) vi[i] = v0[i];
      } else {
        T dv[NV];
#pragma unroll
        for (int i = 0; i < NV; i++) { dv[i] = a * W.vi[i]; vi[i] = v0[i] + h * a * warm[i]; }  // W.vi: previous stage
        integrate_pos(qi, dv, h);
      }
      team_sync();
#pragma unroll
      for (int i = 0; i < NQ; i++) W.u.pre.qi[i] = qi[i];
#pragma unroll
      for (int i = 0; i < NV; i++) W.vi[i] = vi[i];
    }
    // the solve's warm start / result in registers for this forward only
    // (warm may live in the workspace, see step_kernel)
    T acc[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) acc[i] = warm[i];
    if (stage == 3) {
      // stage 4 (t + h) from stage 3 (t + h/2) and stage 1 (t): linear
      // extrapolation in time, 2 k3 - k1.  Only the solver's starting point:
      // the minimiser is unique, so qacc is the same to the solver tolerance;
      // it takes 44% fewer Newton iterations at this stage than k3 itself
      // (tools/solver_stats, flat, random actions).
#pragma unroll
      for (int i = 0; i < NV; i++) acc[i] = 2 * warm[i] - W.k1[i];
    }
    const int fit = forward<T, BODY>(m, W.u.pre.qi, W.vi, ctrl, acc, tr, W, stage == 3 ? &so : (StageOut<T>*)nullptr, tm);
    if (fit < 0) return -1;  // fast path aborted (team-uniform)
    if (stage == 0 && !*acc_reset && team_any(tm, vec_bad(acc, NV))) {
      // mj_checkAcc -> mj_resetData + mj_forward (rare: stage 1 again from qpos0)
      team_sync();
#pragma unroll
      for (int i = 0; i < NQ; i++) q0[i] = m.qpos0[i];
#pragma unroll
      for (int i = 0; i < NV; i++) { v0[i] = 0; warm[i] = 0; }
      ctrl[0] = ctrl[1] = ctrl[2] = 0;
      *acc_reset = true;
      iters += fit;
      stage = -1;
      continue;
    }
#pragma unroll
    for (int i = 0; i < NV; i++) warm[i] = acc[i];
    iters += fit;
#if defined(BB_SOLVE_STATS) && !defined(__HIP_DEVICE_COMPILE__)
    g_stage_iters[stage] = fit;
#endif
    const T b = (stage == 0 || stage == 3) ? T(1.0 / 6) : T(1.0 / 3);  // RK4 weights B
    team_sync();
    if (stage == 0) {
#pragma unroll
      for (int i = 0; i < NV; i++) { vs[i] = b * W.vi[i]; as[i] = b * warm[i]; W.k1[i] = warm[i]; }
    } else {
#pragma unroll
      for (int i = 0; i < NV; i++) { vs[i] += b * W.vi[i]; as[i] += b * warm[i]; }
    }
  }
  team_sync();
  // mj_advance: qvel = v0 + h*qacc_rk ; qpos = q0 (+) h*v_rk
#pragma unroll
  for (int i = 0; i < NV; i++) v[i] = v0[i] + h * as[i];
#pragma unroll
  for (int i = 0; i < NQ; i++) q[i] = q0[i];
  T vv[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) vv[i] = vs[i];
  integrate_pos(q, vv, h);
  return iters;
}

// mj_resetData + height offset (ballbot_env.py:612-620)
template <typename T>
BB_HD void reset_state(const ModelT<T>& m, T offset, T* q, T* v, T* warm) {
#pragma unroll
  for (int i = 0; i < NQ; i++) q[i] = m.qpos0[i];
  q[2] += offset;
  q[12] += offset;
#pragma unroll
  for (int i = 0; i < NV; i++) { v[i] = 0; warm[i] = 0; }
}

// numpy-quaternion as_rotation_vector (quaternion_log, eps 1e-14): no w>=0
// canonicalisation.
template <typename T>
BB_HD void quat_to_rotvec(const T* q, T* rv) {
  T b = sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (fabs(b) <= T(1e-14) * fabs(q[0])) {
    rv[0] = q[0] < 0 ? T(2 * 3.14159265358979323846) : T(0);
    rv[1] = rv[2] = 0;
    return;
  }
  T f = 2 * atan2(b, q[0]) / b;
  rv[0] = f * q[1]; rv[1] = f * q[2]; rv[2] = f * q[3];
}

BB_HD float clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// mj_checkPos / mj_checkVel: NaN or |x| > 1e10 anywhere in qpos or qvel
template <typename T>
BB_HD bool state_bad(const T* q, const T* v) {
  return vec_bad(q, NQ) || vec_bad(v, NV);
}

// flags returned by env_step; F_SLOWPATH: the fast kernel left this env to
// the full kernel (nothing was stepped).  F_DIVERGED: MuJoCo's divergence
// auto-reset ran inside this step (mj_checkPos/Vel/Acc -> mj_resetData); it is
// information, not an episode end: the reference's episode goes on from qpos0
// (ballbot_env.py:897-899 never fires, mj_step advances time past 0).
// F_SPILL (internal): the last RK stage stored base-tree contacts past the
// team's MAXB_LDS LDS slots, in the env's HBM spill block.
constexpr int F_TERMINATED = 1, F_FAILURE = 2, F_DIVERGED = 4, F_OVERFLOW = 8, F_SPILL = 1 << 9,
              F_SLOWPATH = 1 << 16;

// One BBotSimulation.step.  obs15 = sorted keys (actions, angular_vel,
// motor_state, orientation, vel), the order the policy's Extractor consumes.
template <typename T, bool BODY = true>
BB_HD int env_step(const ModelT<T>& m, const EnvCfg& cfg, T* q, T* v, T* warm, int& step, const float* action,
                   const TerrainRef<T>& tr, EnvWork<T>& W, float* obs15, float& reward, float* pos2d,
                   int* iters, const Team& tm) {
  const float mwv = cfg.max_wheel_velocity;
  T ctrl[3];
#pragma unroll
  for (int i = 0; i < 3; i++) ctrl[i] = -T(clipf(action[i] * mwv, -mwv, mwv));  // data.ctrl[:] = -ctrl
  // mjWARN_BADCTRL (mj_fwdActuation): a bad control zeroes all of them
  if (vec_bad(ctrl, 3)) ctrl[0] = ctrl[1] = ctrl[2] = 0;
  int flags = 0;
  // mj_step's mj_checkPos / mj_checkVel: a bad state is mj_resetData'd (qpos0
  // without the reset height offset, zero velocity, warm start and ctrl) and
  // this step integrates from there; step_counter goes on (team-uniform: the
  // state is the team's shared copy)
  if (state_bad(q, v)) {
    reset_state(m, T(0), q, v, warm);
    ctrl[0] = ctrl[1] = ctrl[2] = 0;
    flags = F_DIVERGED;
  }
  StageOut<T>& so = W.so;  // team-shared (LDS): not register-resident across the solves
  bool acc_reset = false;
  int it = rk4_step<T, BODY>(m, q, v, warm, ctrl, tr, W, so, tm, &acc_reset);
  if (it < 0) return F_SLOWPATH;
  if (iters) *iters = it;
  if (acc_reset) flags |= F_DIVERGED;
  if (so.overflow) flags |= F_OVERFLOW;
  if (so.nb > MAXB_LDS) flags |= F_SPILL;
  {
  // obs, reward and termination without FMA contraction: numpy's float32 /
  // float64 chains do not fuse, and every kernel that inlines this (step,
  // multi-step, rollout) then rounds alike
#pragma clang fp contract(off)
  // _get_obs
  T rv[3];
  quat_to_rotvec(so.quat_b, rv);
  float orient[3] = {float(rv[0]), float(rv[1]), float(rv[2])};
  float vel[3], angv[3], motor[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    vel[i] = clipf(float(so.w_world[i]), -2.f, 2.f);     // "vel" = cvel[0:3] (angular)
    angv[i] = clipf(float(so.v_com[i]), -2.f, 2.f);      // "angular_vel" = cvel[3:6] (linear)
    motor[i] = clipf(float(v[1 + i]) / mwv, -2.f, 2.f);  // qvel[joint id 1..3]
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    obs15[i] = action[i]; obs15[3 + i] = angv[i]; obs15[6 + i] = motor[i];
    obs15[9 + i] = orient[i]; obs15[12 + i] = vel[i];
  }
  pos2d[0] = float(so.pb[0]);
  pos2d[1] = float(so.pb[1]);
  // reward terms in float32 (numpy float32 chain under NumPy 2)
  float r;
  if (cfg.reward_kind == 0) {
    r = (vel[0] * cfg.target[0] + vel[1] * cfg.target[1]) * cfg.reward_scale;
  } else if (cfg.reward_kind == 1) {
    float dx = cfg.goal[0] - pos2d[0], dy = cfg.goal[1] - pos2d[1];
    r = (-cfg.goal_scale * sqrtf(dx * dx + dy * dy)) * cfg.reward_scale;
  } else {
    r = 0.f;
  }
  float nrm = sqrtf(action[0] * action[0] + action[1] * action[1] + action[2] * action[2]);
  r = r + cfg.action_reg_coef * (nrm * nrm);
  step += 1;
  if (step >= cfg.max_ep_steps) flags |= F_TERMINATED;
  // tilt: R(from_rotation_vector(f32 rotvec))[2,2]
  T rx = orient[0], ry = orient[1], rz = orient[2];
  T th = sqrt(rx * rx + ry * ry + rz * rz) * T(0.5);
  T sf = th > T(1e-14) ? sin(th) / th : T(1);
  T qw = th > T(1e-14) ? cos(th) : T(1);
  T qx = sf * rx * T(0.5), qy = sf * ry * T(0.5), qz = sf * rz * T(0.5);
  T nn = qw * qw + qx * qx + qy * qy + qz * qz;
  T R22 = T(1) - 2 * (qx * qx + qy * qy) / nn;
  T ang = acos(clampT(R22, T(-1), T(1))) * T(180 / 3.14159265358979323846);
  // a host-side plugin (reward_kind 2) gets the action penalty only: the host
  // adds plugin * scale first and the bonus last, the reference's order
  // (reward_obj(obs) * scale + action_reg, then + survival_bonus)
  if (ang > T(cfg.max_allowed_tilt)) flags |= F_FAILURE | F_TERMINATED;
  else if (cfg.reward_kind != 2) r = r + cfg.survival_bonus;
  reward = r;
  return flags;
  }
}

}  // namespace bb
