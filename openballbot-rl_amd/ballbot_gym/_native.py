"""ctypes binding of the C-ABI library (include/ballbot_mi355x.h).

The HIP library is the only compute path: there is no CPU fallback.  If the
shared object is missing or fails to load, `lib()` raises NativeLibraryError.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "_lib" / "libbb_mi355x.so"
CSRC = PKG.parent / "csrc"
INCLUDE = PKG.parent.parent / "include"

NQ, NV, NOBS, HF_N = 17, 15, 15, 293
DONE_TERMINATED, DONE_FAILURE, DONE_DIVERGED, DONE_OVERFLOW = 1, 2, 4, 8
NSTATS = 8  # BB_NSTATS
REWARD_DIRECTIONAL, REWARD_DISTANCE, REWARD_NONE = 0, 1, 2
DSBL_PASSIVE, DSBL_GRAVITY = 32, 64  # bb_params.opt_disableflags (MuJoCo mjtDisableBit values)


class NativeLibraryError(RuntimeError):
    pass


class BBParams(C.Structure):
    _fields_ = [
        ("max_ep_steps", C.c_int),
        ("max_allowed_tilt", C.c_float),
        ("max_wheel_velocity", C.c_float),
        ("reward_scale", C.c_float),
        ("action_reg_coef", C.c_float),
        ("survival_bonus", C.c_float),
        ("target_dir", C.c_float * 2),
        ("reward_kind", C.c_int),
        ("goal", C.c_float * 2),
        ("goal_scale", C.c_float),
        ("n_terrains", C.c_int),
        ("seed", C.c_uint64),
        ("fp64", C.c_int),
        ("solver_maxiter", C.c_int),
        ("solver_tol", C.c_double),
        ("opt_timestep", C.c_double),
        ("opt_disableflags", C.c_int),
    ]


class PerlinCfg(C.Structure):
    """bb_perlin_cfg (include/ballbot_mi355x.h): terrain/perlin.py:8-16 arguments."""
    _fields_ = [
        ("scale", C.c_double),
        ("octaves", C.c_int),
        ("persistence", C.c_float),
        ("lacunarity", C.c_float),
        ("amplitude", C.c_double),
    ]


class PPOMlpArgs(C.Structure):
    """bb_ppo_mlp_args (include/ballbot_mi355x.h)."""
    _fields_ = [(name, C.c_void_p) for name in ("params", "grad", "exp_avg", "exp_avg_sq")] + [
        ("n_params", C.c_int64),
        ("offsets", C.c_int32 * 21),
    ] + [(name, C.c_void_p) for name in ("obs", "actions", "old_logp", "advantages", "returns", "perm",
                                         "mb_counter", "row_counter", "log", "clip", "lr", "step", "coef")] + [
        ("B", C.c_int32),
        ("normalize_advantage", C.c_int32),
        ("obs_dim", C.c_int32),
        ("obs_direct", C.c_int32),
        ("ent_coef", C.c_float),
        ("vf_coef", C.c_float),
    ] + [(name, C.c_double) for name in ("beta1", "beta2", "eps", "weight_decay", "max_grad_norm")] + [
        ("workspace", C.c_void_p),
        ("workspace_bytes", C.c_int64),
        ("phase", C.c_int32),
        ("adv_stats", C.c_void_p),
    ]


class RolloutArgs(C.Structure):
    """bb_rollout_args (include/ballbot_mi355x.h): one whole PPO rollout in one launch."""
    _fields_ = [
        ("params", C.c_void_p),
        ("offsets", C.c_int32 * 21),
        ("n_params", C.c_int64),
        ("noise", C.c_void_p),
        ("n_steps", C.c_int32),
    ] + [(name, C.c_void_p) for name in ("obs", "last_starts", "ep_ret", "ep_len", "buf_obs", "buf_actions",
                                         "buf_values", "buf_log_prob", "buf_rewards", "buf_starts", "ep_r_out",
                                         "ep_l_out")]


ENCODER_FIELDS = ("conv1_w", "conv1_b", "bn1_w", "bn1_b", "bn1_mean", "bn1_var", "bn1_count",
                  "conv2_w", "conv2_b", "bn2_w", "bn2_b", "bn2_mean", "bn2_var", "bn2_count",
                  "fc_w", "fc_b", "bn3_w", "bn3_b", "bn3_mean", "bn3_var", "bn3_count")


class EncoderParams(C.Structure):
    """bb_encoder_params (include/ballbot_mi355x.h): device pointers of the encoder's tensors."""
    _fields_ = [(name, C.c_void_p) for name in ENCODER_FIELDS]


EXPORTS = [
    "bb_abi_version", "bb_last_error", "bb_default_params", "bb_create", "bb_destroy", "bb_set_hfield",
    "bb_assign_terrain", "bb_reset", "bb_step", "bb_get_state", "bb_set_state", "bb_forward", "bb_get_stats",
    "bb_get_offsets", "bb_get_config", "bb_time_kernel", "bb_kernel_ms", "bb_generate_perlin", "bb_get_hfield",
    "bb_gae", "bb_render_depth", "bb_ppo_loss", "bb_adamw_clip", "bb_ppo_mlp_workspace_bytes", "bb_ppo_mlp_step",
    "bb_ppo_mlp_act", "bb_rollout_track", "bb_depth_encoder_workspace_bytes", "bb_depth_encoder",
    "bb_set_terrain_stream", "bb_get_env_terrain", "bb_kernel_times", "bb_step_multi", "bb_rollout",
    "bb_set_terrain_rng", "bb_get_terrain_rng", "bb_pair_counters", "bb_pair_env_times", "bb_check",
]

ABI_VERSION = 19  # include/ballbot_mi355x.h BB_ABI_VERSION

_lib = None


HIP_SOURCES = ("bb_kernels.hip", "bb_pair.hip", "bb_terrain.hip", "bb_rollout.hip", "bb_render.hip", "bb_ppo.hip",
               "bb_mlp.hip", "bb_encoder.hip")
# per-source flags: the relief pair's unit without MachineLICM (bb_kernels.hip: bb_pair_launch_tu)
SOURCE_FLAGS = {"bb_pair.hip": ["-mllvm", "-disable-machine-licm"]}


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile csrc/*.hip (HIP_SOURCES) for gfx950 into _lib/libbb_mi355x.so: one
    hipcc -c per source, in parallel (objects under _lib/obj), then one link."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor

    srcs = list(CSRC.glob("*.h")) + list(CSRC.glob("*.hip")) + list(INCLUDE.glob("*.h"))
    if LIB_PATH.exists() and not force and all(LIB_PATH.stat().st_mtime >= s.stat().st_mtime for s in srcs):
        return LIB_PATH
    obj_dir = LIB_PATH.parent / "obj"
    obj_dir.mkdir(parents=True, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC"]
    jobs = []
    for f in HIP_SOURCES:
        obj = obj_dir / (f[:-4] + ".o")
        jobs.append((["hipcc", *flags, *SOURCE_FLAGS.get(f, []), "-c", "-o", str(obj), str(CSRC / f)], obj))
    if verbose:
        for cmd, _ in jobs:
            print(" ".join(cmd))

    def run(job):
        return subprocess.run(job[0], capture_output=True, text=True)

    workers = max(1, min(len(jobs), os.cpu_count() or 1, 16))
    with ThreadPoolExecutor(workers) as ex:
        results = list(ex.map(run, jobs))
    for (cmd, _), r in zip(jobs, results):
        if r.returncode != 0:
            raise subprocess.CalledProcessError(r.returncode, cmd, r.stdout, r.stderr + "\n" + " ".join(cmd))
    tmp = LIB_PATH.with_suffix(".so.tmp")
    link = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *[str(o) for _, o in jobs]]
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def lib():
    """The product library (csrc/bb_kernels.hip built for gfx950); raises if absent."""
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


def use_diagnostic_library(path) -> None:
    """Load an instrumented build of the same sources (tools/ only, e.g. -DBB_PHASE_CLOCKS)."""
    global _lib
    _lib = _load(Path(path))


def _load(path: Path):
    if not path.exists():
        raise NativeLibraryError(
            f"HIP library {path} not found; run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    try:
        L = C.CDLL(str(path))
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load {path}: {e}") from e
    vp, fp, dp = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_double)
    L.bb_abi_version.restype = C.c_int
    L.bb_last_error.argtypes = [C.c_char_p, C.c_int]
    L.bb_default_params.argtypes = [C.POINTER(BBParams)]
    L.bb_default_params.restype = None
    L.bb_create.argtypes = [C.c_int, C.c_int, C.POINTER(BBParams), C.POINTER(vp)]
    L.bb_destroy.argtypes = [vp]
    L.bb_set_hfield.argtypes = [vp, C.c_int, fp, C.c_float]
    L.bb_assign_terrain.argtypes = [vp, vp, vp]
    L.bb_reset.argtypes = [vp, vp, vp, vp]
    L.bb_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, C.c_int, vp]
    L.bb_step_multi.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp]
    L.bb_rollout.argtypes = [vp, C.POINTER(RolloutArgs), vp]
    L.bb_get_state.argtypes = [vp, dp, dp, dp, C.POINTER(C.c_int32)]
    L.bb_set_state.argtypes = [vp, dp, dp, dp, C.POINTER(C.c_int32)]
    L.bb_forward.argtypes = [vp, dp, dp, C.POINTER(C.c_int32)]
    L.bb_get_stats.argtypes = [vp, C.POINTER(C.c_int64), C.c_int]
    L.bb_pair_counters.argtypes = [vp, C.POINTER(C.c_int64), C.c_int]
    L.bb_pair_env_times.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.bb_check.argtypes = [vp, vp]
    L.bb_set_terrain_stream.argtypes = [vp, C.POINTER(C.c_int32), C.c_int, C.c_int, C.POINTER(C.c_int32)]
    L.bb_set_terrain_rng.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]
    L.bb_get_terrain_rng.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]
    L.bb_get_env_terrain.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.bb_get_offsets.argtypes = [vp, fp]
    L.bb_get_config.argtypes = [vp, C.POINTER(C.c_int32)]
    L.bb_time_kernel.argtypes = [vp, C.c_int]
    L.bb_generate_perlin.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_int32), C.POINTER(PerlinCfg), C.c_float]
    L.bb_get_hfield.argtypes = [vp, C.c_int, fp]
    L.bb_render_depth.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    L.bb_ppo_loss.argtypes = [vp] * 8 + [C.c_int, C.c_int, C.c_float, C.c_float, vp, vp, vp, vp]
    L.bb_adamw_clip.argtypes = [vp, vp, vp, vp, C.c_int64, vp, vp, vp] + [C.c_double] * 5 + [vp]
    L.bb_gae.argtypes = [vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_double, C.c_double, vp, vp, vp]
    L.bb_ppo_mlp_workspace_bytes.argtypes = [C.c_int, C.POINTER(C.c_int64)]
    L.bb_ppo_mlp_step.argtypes = [C.POINTER(PPOMlpArgs), vp]
    L.bb_ppo_mlp_act.argtypes = [vp, C.POINTER(C.c_int32), C.c_int64, vp, C.c_int, vp, C.c_int, vp, vp, vp, vp, vp,
                                 vp]
    L.bb_rollout_track.argtypes = [vp, vp, C.c_int, C.c_int] + [vp] * 8
    L.bb_depth_encoder_workspace_bytes.argtypes = [C.c_int64, C.POINTER(C.c_int64)]
    L.bb_depth_encoder.argtypes = [C.POINTER(EncoderParams), vp, C.c_int64, vp, C.c_int64, C.c_int, C.c_int, C.c_int,
                                   C.c_float, C.c_float, vp, C.c_int64, vp, C.c_int64, vp]
    L.bb_kernel_ms.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    L.bb_kernel_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    for name in [n for n in EXPORTS if n not in ("bb_default_params", "bb_abi_version")]:
        getattr(L, name).restype = C.c_int
    if L.bb_abi_version() != ABI_VERSION:
        raise NativeLibraryError("ABI version mismatch")
    return L


def last_error() -> str:
    buf = C.create_string_buffer(512)
    lib().bb_last_error(buf, 512)
    return buf.value.decode()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {last_error()}")


def default_params() -> BBParams:
    p = BBParams()
    lib().bb_default_params(C.byref(p))
    return p
