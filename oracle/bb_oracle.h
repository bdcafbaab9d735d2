/*
 * bb_oracle.h -- CPU fp64 restatement of the reference's `mj_step` hot path for
 * ballbot.xml, plus the env step glue of ballbot_gym/envs/ballbot_env.py.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (openballbot-rl_amd/csrc) never links or calls it.
 *
 * Parity status
 *   - physics (A3..A9 of SURVEY.md §8): UNPINNED against real MuJoCo.  MuJoCo
 *     (git 99490163 + tools/mujoco_fix.patch) is not vendored in the reference
 *     and cannot be built or imported here.  This file restates MuJoCo's
 *     published algorithms for this one model; it is validated by physical
 *     invariants (tests/test_oracle.py: free fall, energy and momentum
 *     conservation, mass-matrix structure, patched contact frame, PID balance).
 *   - glue (A10..A15): the reward chain is checked against the reward plugin
 *     pinned by golden vectors from the reference's importable Python modules
 *     (tests/golden/, tools/gen_goldens.py); obs packing (numpy-quaternion
 *     rotvec) and termination are restated from ballbot_env.py:771-1036 and
 *     formula-pinned (no MuJoCo run can produce reference outputs here).
 *
 * All state is MuJoCo layout: qpos[17] = base(x,y,z,qw,qx,qy,qz), wheel0..2,
 * ball(x,y,z,qw,qx,qy,qz); qvel[15] = base(v_world[3], w_local[3]),
 * wheel0..2 rates, ball(v_world[3], w_local[3]).
 */
#ifndef BB_ORACLE_H
#define BB_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define BBO_NQ 17
#define BBO_NV 15
#define BBO_NU 3
#define BBO_NBODY 8
#define BBO_HF_N 293          /* ballbot.xml:23 nrow = ncol = 293 */
#define BBO_MAXGROUND 50      /* cap on ball-hfield contacts = MuJoCo mjMAXCONPAIR */
#define BBO_MAXPAIR 50        /* contacts per hfield x geom pair = MuJoCo mjMAXCONPAIR (first 50 in prism order) */
/* base-tree geom contacts: ball x {tower, sticks} (one each) + hfield x {tower, sticks, wheels} */
#define BBO_MAXBODY (3 + 6 * BBO_MAXPAIR)
#define BBO_MAXCON (3 + BBO_MAXGROUND + BBO_MAXBODY)

/* option flags for invariant tests (0 = reference behaviour) */
#define BBO_DISABLE_CONTACT 1
#define BBO_DISABLE_GRAVITY 2
#define BBO_DISABLE_DAMPING 4
/* test-only: compose the free joints' rotations in RK4 as Runge-Kutta-Munthe-Kaas
 * (stage rates dexp^-1 of the body angular velocity, relative to the step's start
 * orientation) instead of MuJoCo's sum of the stages' body-frame angular velocities.
 * Pins that the forward dynamics are consistent to 4th order (tests/test_oracle.py). */
#define BBO_RKMK 8
/* test-only: start every solve from qacc_warmstart, without MuJoCo's comparison against
 * qacc_smooth (the kernel's start; DESIGN.md §4 measures the difference) */
#define BBO_WARM_ONLY 16

/* Per-forward diagnostic outputs (stage-level view of mjData). */
typedef struct {
  double qacc[BBO_NV];
  double qacc_smooth[BBO_NV];
  double qfrc_bias[BBO_NV];
  double M[BBO_NV * BBO_NV];
  double xpos_base[3], xquat_base[4];
  double cvel_base[6];          /* MuJoCo cvel[base]: [w_world; v at subtree_com] */
  double subtree_com_base[3];
  int ncon, nground, niter;
  double con_dist[BBO_MAXCON];
  double con_pos[BBO_MAXCON * 3];
  double con_frame[BBO_MAXCON * 9];
  int con_body2[BBO_MAXCON];    /* 4..6 = wheel (ball is geom1), 7 = ball vs hfield */
  double energy_kin, energy_pot;
  int ground_overflow;          /* bit 0: ball-hfield cap, bit 1: base-tree contact cap */
  int nbody;                    /* base-tree geom contacts (after the 3 wheel + nground ball contacts) */
  int con_body1[BBO_MAXCON];    /* 0 world (hfield), 7 ball */
  double con_force[BBO_MAXCON * 3];  /* efc_force per contact: normal, tangent 1, tangent 2 (contact frame) */
} bbo_forward_out;

/* Env configuration mirroring BBotSimulation.__init__ (ballbot_env.py:157-231). */
typedef struct {
  int max_ep_steps;             /* default 4000 */
  double max_allowed_tilt;      /* degrees, default 20 */
  double max_wheel_velocity;    /* default 10 */
  float reward_scale;           /* 0.01 */
  float action_reg_coef;        /* -1e-4 */
  float survival_bonus;         /* 0.02 */
  float target_dir[2];          /* DirectionalReward target (0, 1) */
} bbo_env_cfg;

/* Model/options.  size_z: hfield size[2] (ballbot.xml:23, 2.0; ramp/gradient rescale). */
int  bbo_abi_version(void);
void bbo_set_flags(int flags);
int  bbo_get_flags(void);
void bbo_set_solver(int maxiter, double tol);
/* line search: at most ls_iterations evaluations, stop at |phi'| <= ls_tolerance |phi'(0)| */
void bbo_set_linesearch(int ls_iterations, double ls_tolerance);
void bbo_model_info(double* out);
/* opt.timestep (invariant tests: RK4 order; h <= 0 restores 0.002) */
void bbo_set_timestep(double h);
/* momentum of the bodies at (qpos, qvel): out[0..3) linear, out[3..6) angular about
 * the system COM (world frame), out[6..9) the system COM */
void bbo_momentum(const double* qpos, const double* qvel, double* out);   /* masses, invweight0, meaninertia, qpos0 ... (see .c) */

/* mj_forward at (qpos, qvel) with ctrl; warm = qacc_warmstart (may be NULL). */
void bbo_forward(const double* qpos, const double* qvel, const double* ctrl,
                 const double* warm, const float* hfield, double size_z,
                 bbo_forward_out* out);

/* mj_step with RK4: advances qpos/qvel/warm in place.  stage4 (may be NULL)
 * receives the forward outputs of the last RK stage (what mjData holds after
 * mj_step: xquat/cvel/xpos come from RK stage 4).  MuJoCo's
 * divergence handling is restated: a NaN/|x|>1e10 qpos or qvel (mj_checkPos/
 * Vel) or qacc after the first forward (mj_checkAcc) resets to qpos0 with zero
 * velocity, warm start and ctrl, and the step integrates from there; a bad
 * ctrl zeroes all ctrl (mjWARN_BADCTRL).  Returns 1 if such a reset happened. */
int bbo_mj_step(double* qpos, double* qvel, double* warm, const double* ctrl,
                 const float* hfield, double size_z, bbo_forward_out* stage4);

/* Full env step (ballbot_env.py:854-1036) for one env.
 * obs15 layout = sorted keys: actions, angular_vel, motor_state, orientation, vel.
 * Returns flags: bit0 terminated, bit1 failure (tilt), bit2 diverged. */
int bbo_env_step(const bbo_env_cfg* cfg, double* qpos, double* qvel, double* warm,
                 int* step_counter, const float* action, const float* hfield,
                 double size_z, float* obs15, float* reward, float* pos2d,
                 double* tilt_deg);

/* Reset state (ballbot_env.py:612-620): qpos0 with height offset, zero vel. */
void bbo_reset_state(double offset, double* qpos, double* qvel, double* warm);

/* init height offset of _reset_terrain (ballbot_env.py:527-565), incl. its
 * cell_size = size/nrows quirk. */
double bbo_init_offset(const float* hfield, double size_z);

/* numpy-quaternion as_rotation_vector restatement (quaternion_log). */
void bbo_quat_to_rotvec(const double* q, double* rv);

/* Depth image of cam (0/1) at qpos: float32[H][W], linear z-depth clipped to 1
 * (sensors/rgbd.py:46-82 over ballbot.xml:44-54; see bb_oracle.c). */
void bbo_render_depth(const double* qpos, const float* hfield, double size_z, int cam, int H, int W, float* out);

/* Batch helper: n envs stepped sequentially on one thread (CPU baseline). */
int bbo_env_step_batch(const bbo_env_cfg* cfg, int n, double* qpos, double* qvel,
                       double* warm, int* step_counter, const float* actions,
                       const float* hfield, double size_z, float* obs,
                       float* reward, unsigned char* done, double offset);

/* bbo_env_step_batch with one env per OpenMP thread (threads >= 1). */
int bbo_env_step_batch_mt(const bbo_env_cfg* cfg, int n, double* qpos, double* qvel, double* warm,
                          int* step_counter, const float* actions, const float* hfield, double size_z,
                          float* obs, float* reward, unsigned char* done, double offset, int threads);

#ifdef __cplusplus
}
#endif
#endif
