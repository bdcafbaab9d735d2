"""ctypes binding of the CPU fp64 oracle (oracle/bb_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker, never as the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
LIB_PATH = ORACLE_DIR / "_build" / "libbb_oracle.so"

NQ, NV, NB, MAXCON = 17, 15, 8, 356  # MAXCON = 3 + BBO_MAXGROUND 50 + BBO_MAXBODY (3 + 6 x 50)
HF_N = 293

DISABLE_CONTACT, DISABLE_GRAVITY, DISABLE_DAMPING, RKMK, WARM_ONLY = 1, 2, 4, 8, 16


class ForwardOut(C.Structure):
    _fields_ = [
        ("qacc", C.c_double * NV),
        ("qacc_smooth", C.c_double * NV),
        ("qfrc_bias", C.c_double * NV),
        ("M", C.c_double * (NV * NV)),
        ("xpos_base", C.c_double * 3),
        ("xquat_base", C.c_double * 4),
        ("cvel_base", C.c_double * 6),
        ("subtree_com_base", C.c_double * 3),
        ("ncon", C.c_int),
        ("nground", C.c_int),
        ("niter", C.c_int),
        ("con_dist", C.c_double * MAXCON),
        ("con_pos", C.c_double * (MAXCON * 3)),
        ("con_frame", C.c_double * (MAXCON * 9)),
        ("con_body2", C.c_int * MAXCON),
        ("energy_kin", C.c_double),
        ("energy_pot", C.c_double),
        ("ground_overflow", C.c_int),
        ("nbody", C.c_int),
        ("con_body1", C.c_int * MAXCON),
        ("con_force", C.c_double * (MAXCON * 3)),
    ]


class EnvCfg(C.Structure):
    _fields_ = [
        ("max_ep_steps", C.c_int),
        ("max_allowed_tilt", C.c_double),
        ("max_wheel_velocity", C.c_double),
        ("reward_scale", C.c_float),
        ("action_reg_coef", C.c_float),
        ("survival_bonus", C.c_float),
        ("target_dir", C.c_float * 2),
    ]


def default_cfg(max_ep_steps=4000, target=(0.0, 1.0)) -> EnvCfg:
    cfg = EnvCfg()
    cfg.max_ep_steps = max_ep_steps
    cfg.max_allowed_tilt = 20.0
    cfg.max_wheel_velocity = 10.0
    cfg.reward_scale = 0.01
    cfg.action_reg_coef = -0.0001
    cfg.survival_bonus = 0.02
    cfg.target_dir[0], cfg.target_dir[1] = target
    return cfg


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        dp, fp, ip = C.POINTER(C.c_double), C.POINTER(C.c_float), C.POINTER(C.c_int)
        L.bbo_forward.argtypes = [dp, dp, dp, dp, fp, C.c_double, C.POINTER(ForwardOut)]
        L.bbo_mj_step.argtypes = [dp, dp, dp, dp, fp, C.c_double, C.POINTER(ForwardOut)]
        L.bbo_env_step.argtypes = [C.POINTER(EnvCfg), dp, dp, dp, ip, fp, fp, C.c_double, fp, fp, fp, dp]
        L.bbo_env_step.restype = C.c_int
        L.bbo_reset_state.argtypes = [C.c_double, dp, dp, dp]
        L.bbo_init_offset.argtypes = [fp, C.c_double]
        L.bbo_init_offset.restype = C.c_double
        L.bbo_quat_to_rotvec.argtypes = [dp, dp]
        L.bbo_model_info.argtypes = [dp]
        L.bbo_set_flags.argtypes = [C.c_int]
        L.bbo_set_solver.argtypes = [C.c_int, C.c_double]
        L.bbo_env_step_batch.argtypes = [C.POINTER(EnvCfg), C.c_int, dp, dp, dp, ip, fp, fp, C.c_double,
                                         fp, fp, C.POINTER(C.c_ubyte), C.c_double]
        L.bbo_env_step_batch.restype = C.c_int
        L.bbo_env_step_batch_mt.argtypes = L.bbo_env_step_batch.argtypes + [C.c_int]
        L.bbo_env_step_batch_mt.restype = C.c_int
        L.bbo_render_depth.argtypes = [dp, fp, C.c_double, C.c_int, C.c_int, C.c_int, fp]
        L.bbo_set_timestep.argtypes = [C.c_double]
        L.bbo_momentum.argtypes = [dp, dp, dp]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


def flat_hfield() -> np.ndarray:
    return np.zeros(HF_N * HF_N, dtype=np.float32)


def model_info() -> dict:
    out = np.zeros(64)
    lib().bbo_model_info(_d(out))
    return {
        "mass": out[0:8].copy(),
        "invweight_tran": out[8:16].copy(),
        "invweight_rot": out[16:24].copy(),
        "meaninertia": float(out[24]),
        "qpos0": out[25:42].copy(),
        "wheel0_ipos": out[42:45].copy(),
        "base_inertia": out[45:54].reshape(3, 3).copy(),
    }


def render_depth(qpos: np.ndarray, hfield: np.ndarray, cam: int, H: int = 64, W: int = 64,
                 size_z: float = 2.0) -> np.ndarray:
    """Depth image float32[H, W] of cam 0/1 (bbo_render_depth)."""
    out = np.zeros((H, W), np.float32)
    q = np.ascontiguousarray(qpos, np.float64)
    lib().bbo_render_depth(_d(q), _f(np.ascontiguousarray(hfield, np.float32)), float(size_z), int(cam), H, W, _f(out))
    return out


def set_flags(flags: int) -> None:
    lib().bbo_set_flags(flags)


def set_timestep(h: float = 0.002) -> None:
    """opt.timestep of the oracle's mj_step (the RK4 convergence test)."""
    lib().bbo_set_timestep(float(h))


def momentum(qpos, qvel):
    """(linear momentum, angular momentum about the system COM, system COM) of the bodies."""
    out = np.zeros(9)
    lib().bbo_momentum(_d(np.ascontiguousarray(qpos, np.float64)), _d(np.ascontiguousarray(qvel, np.float64)), _d(out))
    return out[0:3], out[3:6], out[6:9]


def set_solver(maxiter: int = 100, tol: float = 1e-12) -> None:
    lib().bbo_set_solver(maxiter, tol)


def reset_state(offset: float = 0.01):
    q = np.zeros(NQ)
    v = np.zeros(NV)
    w = np.zeros(NV)
    lib().bbo_reset_state(offset, _d(q), _d(v), _d(w))
    return q, v, w


def init_offset(hfield: np.ndarray, size_z: float = 2.0) -> float:
    hf = np.ascontiguousarray(hfield, dtype=np.float32)
    return lib().bbo_init_offset(_f(hf), size_z)


def forward(qpos, qvel, ctrl=None, warm=None, hfield=None, size_z=2.0) -> ForwardOut:
    out = ForwardOut()
    q = np.ascontiguousarray(qpos, dtype=np.float64)
    v = np.ascontiguousarray(qvel, dtype=np.float64)
    c = None if ctrl is None else np.ascontiguousarray(ctrl, dtype=np.float64)
    w = None if warm is None else np.ascontiguousarray(warm, dtype=np.float64)
    hf = None if hfield is None else np.ascontiguousarray(hfield, dtype=np.float32)
    lib().bbo_forward(_d(q), _d(v), None if c is None else _d(c), None if w is None else _d(w), _f(hf), size_z,
                      C.byref(out))
    return out


def mj_step(qpos, qvel, warm, ctrl, hfield=None, size_z=2.0):
    """In-place RK4 mj_step; returns the stage-4 ForwardOut."""
    out = ForwardOut()
    c = np.ascontiguousarray(ctrl, dtype=np.float64)
    hf = None if hfield is None else np.ascontiguousarray(hfield, dtype=np.float32)
    lib().bbo_mj_step(_d(qpos), _d(qvel), _d(warm), _d(c), _f(hf), size_z, C.byref(out))
    return out


def env_step(cfg, qpos, qvel, warm, step_counter, action, hfield, size_z=2.0):
    """One BBotSimulation.step on the oracle. Mutates qpos/qvel/warm/step_counter (np int32[1])."""
    obs = np.zeros(15, dtype=np.float32)
    rew = np.zeros(1, dtype=np.float32)
    pos2d = np.zeros(2, dtype=np.float32)
    tilt = np.zeros(1)
    a = np.ascontiguousarray(action, dtype=np.float32)
    hf = np.ascontiguousarray(hfield, dtype=np.float32)
    flags = lib().bbo_env_step(C.byref(cfg), _d(qpos), _d(qvel), _d(warm),
                               step_counter.ctypes.data_as(C.POINTER(C.c_int)), _f(a), _f(hf), size_z,
                               _f(obs), _f(rew), _f(pos2d), _d(tilt))
    return obs, float(rew[0]), flags, pos2d, float(tilt[0])


def quat_to_rotvec(q) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.float64)
    rv = np.zeros(3)
    lib().bbo_quat_to_rotvec(_d(q), _d(rv))
    return rv


def env_step_batch(cfg, qpos, qvel, warm, steps, actions, hfield, size_z, offset, threads=1):
    """Step n envs on the CPU (threads > 1: one env per OpenMP thread)."""
    n = qpos.shape[0]
    obs = np.zeros((n, 15), dtype=np.float32)
    rew = np.zeros(n, dtype=np.float32)
    done = np.zeros(n, dtype=np.uint8)
    hf = np.ascontiguousarray(hfield, dtype=np.float32)
    a = np.ascontiguousarray(actions, dtype=np.float32)
    args = (C.byref(cfg), n, _d(qpos), _d(qvel), _d(warm), steps.ctypes.data_as(C.POINTER(C.c_int)), _f(a), _f(hf),
            size_z, _f(obs), _f(rew), done.ctypes.data_as(C.POINTER(C.c_ubyte)), offset)
    if threads > 1:
        lib().bbo_env_step_batch_mt(*args, int(threads))
    else:
        lib().bbo_env_step_batch(*args)
    return obs, rew, done
