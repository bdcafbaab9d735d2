"""BallbotVecEnv: N ballbot envs stepped by one HIP launch per env.step.

Batched replacement for `BBotSimulation` (ballbot_gym/envs/ballbot_env.py:60)
as driven by SB3's VecEnv (ballbot_rl/training/train.py:60-120): the physics
(`mujoco.mj_step`, ballbot_env.py:912), observation packing (:771-811), the
reward plugin (:929-937) and termination (:982-1017) all run in the fused
step kernel behind the C-ABI (include/ballbot_mi355x.h).  Tensors live on the
GPU; `step` takes and returns torch tensors on `device`.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, Optional, Sequence

import numpy as np
import torch

from .. import _native as N

OBS_KEYS = ("actions", "angular_vel", "motor_state", "orientation", "vel")  # sorted, as the policy reads them


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class BallbotVecEnv:
    """Vectorised ballbot env on one GPU.

    Args mirror BBotSimulation (ballbot_env.py:157-231) plus `num_envs`,
    `device`, `precision` ("fp32" | "fp64") and the terrain bank size.

    Terrain seeds follow the reference's per-reset draw r_seed =
    _np_random.integers(0, 10000) (ballbot_env.py:505-510), drawn on the GPU
    from numpy's PCG64 per env (bb_set_terrain_rng).  By default env i draws
    from np_random(seed + i): SB3 seeds the training VecEnv that way
    (VecEnv.seed(seed), then reset(seed=seed+i) in learn(); gymnasium's
    Env.reset replaces _np_random, ballbot_env.py:596; train.py:126-141).
    `stream_seeds` gives env i np_random(stream_seeds[i]) (an eval VecEnv:
    seed + N_ENVS + i, train.py:90-97); `shared_stream=True` puts every env on
    np_random(seed).  `seed(s)` re-seeds env i to np_random(s + i) at the next
    reset(), as SB3's VecEnv.seed does.  `n_terrains`: the draws per generator
    whose terrains a host-generated bank holds (perlin default: the whole
    10^4-seed space, generated on the GPU).  `terrain_draws`: an explicit list
    of terrain seeds that every env walks instead (a replayed draw log).
    """

    metadata = {"render_modes": []}
    render_mode = None

    def __init__(
        self,
        num_envs: int,
        device: str | torch.device = "cuda:0",
        reward_config: Optional[Dict[str, Any]] = None,
        terrain_config: Optional[Dict[str, Any]] = None,
        env_config: Optional[Dict[str, Any]] = None,
        max_ep_steps: Optional[int] = None,
        seed: int = 0,
        precision: str = "fp64",
        n_terrains: Optional[int] = None,
        auto_reset: bool = True,
        disable_cameras: bool = True,
        stream_seeds: Optional[Sequence[int]] = None,
        terrain_draws: Optional[Sequence[int]] = None,
        shared_stream: bool = False,
        terrain_slots: Optional[int] = None,
        reward_compat: str = "reference",
        opt_timestep: Optional[float] = None,
        opt_disableflags: int = 0,
    ):
        from .config import params_from_configs

        if not torch.cuda.is_available():
            raise RuntimeError("BallbotVecEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError(f"BallbotVecEnv runs on a GPU device, got {self.device}")
        self.num_envs = int(num_envs)
        self.auto_reset = bool(auto_reset)
        # depth cameras (ballbot_env.py:211-290; camera: height/width/frame_rate/disable_rgb).
        # The reference defaults to cameras on; the batched env defaults to off (the
        # proprio hot path) -- pass disable_cameras=False for rgbd_0/rgbd_1 obs.
        self.cameras = not disable_cameras
        cam = ((env_config or {}).get("camera", {}) or {})
        self.cam_h, self.cam_w = int(cam.get("height", 64)), int(cam.get("width", 64))
        fr = float(cam.get("frame_rate", 90))
        self.cam_every = int(np.ceil((1.0 / fr) / float(opt_timestep or 0.002)))  # effective_camera_frame_rate (ballbot_env.py:389-411)
        if self.cameras and not cam.get("disable_rgb", True):
            raise ValueError("only depth cameras are rendered (camera.disable_rgb must be true)")
        self.terrain_config = terrain_config or {"type": "flat", "config": {}}
        self.reward_config = reward_config or {"type": "directional", "config": {"target_direction": [0.0, 1.0]}}
        p, self.reward_obj, self._host_reward = params_from_configs(self.reward_config, env_config, max_ep_steps,
                                                                    precision, seed, reward_compat=reward_compat)
        from .config import reward_error

        # reward_compat="reference": a DistanceReward raises at the first step, as
        # in the reference env (its obs lacks pos2d); "fused": the kernel computes it
        self._reward_error = reward_error(self.reward_obj, reward_compat)
        # mjModel.opt overrides (physics invariant tests): timestep and MuJoCo's
        # mjDSBL_PASSIVE / mjDSBL_GRAVITY bits (_native.DSBL_*); the reference never sets them
        p.opt_timestep = float(opt_timestep or 0.0)
        p.opt_disableflags = int(opt_disableflags)
        self.opt_timestep = float(opt_timestep or 0.002)
        self.max_ep_steps = int(p.max_ep_steps)
        self.precision = "fp64" if p.fp64 else "fp32"
        self._params = p
        self._seed = int(seed)
        self._n_terrains_arg = n_terrains
        self._shared_stream = bool(shared_stream)
        self._pending_seeds: Optional[list] = None
        self._graphs = 0  # HIP graphs captured over this handle (capture_step, the trainer's rollout graph)
        self._h = None
        if terrain_slots is not None:  # host-driven terrains (load_terrain + assign_terrain), e.g. BBotSimulation
            from .config import TerrainPlan, terrain_size_z

            plan = TerrainPlan([-1] * int(terrain_slots), None, None, False, terrain_size_z(self.terrain_config))
            self._install(plan, generate=False)
        else:
            self._install(self._plan(stream_seeds, terrain_draws))
        n, dev = self.num_envs, self.device
        self.obs = torch.zeros(n, N.NOBS, dtype=torch.float32, device=dev)
        self.terminal_obs = torch.zeros(n, N.NOBS, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(n, dtype=torch.float32, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.pos2d = torch.zeros(n, 2, dtype=torch.float32, device=dev)
        if self.cameras:
            self.depth = torch.ones(n, 2, self.cam_h, self.cam_w, dtype=torch.float32, device=dev)
            self.rel_ts = torch.zeros(n, dtype=torch.float32, device=dev)
        from .. import spaces

        # SB3 VecEnv / gymnasium attributes (ballbot_env.py:235-256)
        self.action_space = spaces.action_space()
        self.observation_space = spaces.observation_space({"h": self.cam_h, "w": self.cam_w}, 1, not self.cameras)
        self._pending_actions: Optional[torch.Tensor] = None
        self.reset()  # the first reset: draw 0 of every env's generator

    # ------------------------------------------------------------ terrain bank
    def _plan(self, stream_seeds=None, terrain_draws=None):
        from .config import gpu_perlin_plan, terrain_plan

        gp = gpu_perlin_plan(self.terrain_config, self._n_terrains_arg, self._seed, self.num_envs, stream_seeds,
                             terrain_draws, shared=self._shared_stream)
        if gp is not None:
            return gp[0]
        return terrain_plan(self.terrain_config, self._n_terrains_arg, self._seed, self.num_envs, stream_seeds,
                            draws=terrain_draws, shared=self._shared_stream)

    def _install(self, plan, generate: bool = True) -> None:
        """A handle whose bank holds the plan's terrains, with its generators
        (bb_set_terrain_rng) or draw table (bb_set_terrain_stream) installed."""
        from .config import bank_fields, perlin_cfg

        perlin = self._gpu_perlin()
        bank = []
        if generate and not perlin:
            bank = [(h, plan.size_z) for h in bank_fields(self.terrain_config, plan)]
        p = self._params
        p.n_terrains = len(plan.seeds)
        L = N.lib()
        if self._h is not None:
            if self._graphs:
                raise RuntimeError(
                    f"{self._graphs} HIP graph(s) were captured over this env's handle, and the new terrain "
                    "generators' draws are not in its bank: regenerating the bank needs a new handle, which "
                    "those graphs would not follow (re-seed before capturing, or with a bank that covers the "
                    "new draws, e.g. perlin's whole seed space)")
            L.bb_destroy(self._h)
            self._h = None
        h = C.c_void_p()
        N.check(L.bb_create(self.num_envs, self.device.index or 0, C.byref(p), C.byref(h)), "bb_create")
        self._h = h
        for i, (data, size_z) in enumerate(bank):
            arr = np.ascontiguousarray(data, dtype=np.float32)
            N.check(L.bb_set_hfield(h, i, arr.ctypes.data_as(C.POINTER(C.c_float)), float(size_z)), "bb_set_hfield")
        if generate and perlin:
            sd = np.ascontiguousarray(plan.seeds, dtype=np.int32)
            N.check(L.bb_generate_perlin(h, 0, len(sd), sd.ctypes.data_as(C.POINTER(C.c_int32)),
                                         C.byref(perlin_cfg(self.terrain_config)), float(plan.size_z)),
                    "bb_generate_perlin")
        self.terrain_plan = plan
        self.terrain_seeds = plan.seeds
        self.n_terrains = p.n_terrains
        # any terrain with relief: bb_step routes through the predictor (route 0) on such banks
        self.relief = (generate and perlin) or any(float(np.max(data)) > 0.0 for data, _ in bank)
        self._set_draws(plan)

    def _gpu_perlin(self) -> bool:
        tc = self.terrain_config
        return tc.get("type", "flat") == "perlin" and (tc.get("config", {}) or {}).get("seed") is None

    def _set_draws(self, plan) -> None:
        L, ip = N.lib(), C.POINTER(C.c_int32)
        if plan.stream_seeds is not None:  # one PCG64 per env on the device
            words = np.ascontiguousarray(plan.rng_words())
            ss = None if plan.seed_slot is None else np.ascontiguousarray(plan.seed_slot, dtype=np.int32)
            N.check(L.bb_set_terrain_rng(self._h, words.ctypes.data_as(C.POINTER(C.c_uint64)),
                                         None if ss is None else ss.ctypes.data_as(ip)), "bb_set_terrain_rng")
        elif plan.streams is not None:  # an explicit draw table
            st = np.ascontiguousarray(plan.streams, dtype=np.int32)
            es = None if plan.env_stream is None else np.ascontiguousarray(plan.env_stream, dtype=np.int32)
            N.check(L.bb_set_terrain_stream(self._h, st.ctypes.data_as(ip), st.shape[0], st.shape[1],
                                            None if es is None else es.ctypes.data_as(ip)), "bb_set_terrain_stream")

    def _reseed(self, stream_seeds) -> None:
        """Put env i on np_random(stream_seeds[i]) from its next reset on (its draw
        counter restarts).  The generators are rewritten in place (bb_set_terrain_rng), so
        HIP graphs captured before this draw from them at replay.  A bank that lacks the new
        generators' first draws would need a new handle: refused once graphs exist."""
        from .config import stream_draws, terrain_plan

        plan = self.terrain_plan
        if plan.stream_seeds is None and plan.streams is None:
            return  # one fixed terrain (flat or a config seed): nothing is drawn
        stream_seeds = [int(x) for x in stream_seeds]
        if len(stream_seeds) != self.num_envs:
            raise ValueError(f"need one seed per env ({self.num_envs}), got {len(stream_seeds)}")
        k = self._n_terrains_arg or 8
        need = {int(v) for s in dict.fromkeys(stream_seeds) for v in stream_draws(s, k)}
        if plan.stream_seeds is not None and plan.covers(need):
            from .config import TerrainPlan

            new = TerrainPlan(plan.seeds, stream_seeds, plan.seed_slot, plan.full, plan.size_z, seedless=plan.seedless)
            self.terrain_plan = new
            self._set_draws(new)
            return
        self._install(self._plan(stream_seeds))

    # --------------------------------------------------------------------- api
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, mask: Optional[torch.Tensor] = None):
        """Reset every env (mask None) or the masked ones -> (obs, {}).  A full
        reset first applies the seeds of seed(), as SB3's VecEnv.reset passes
        seed + i to env i's reset (then forgets them)."""
        if mask is None and self._pending_seeds is not None:
            pending, self._pending_seeds = self._pending_seeds, None
            self._reseed(pending)
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        N.check(N.lib().bb_reset(self._h, _ptr(m), _ptr(self.obs), self._stream()), "bb_reset")
        if self.cameras:
            self._render(force=m is None)
        return self.obs, {}

    def _render(self, force: bool) -> None:
        N.check(N.lib().bb_render_depth(self._h, _ptr(self.depth), _ptr(self.rel_ts), self.cam_h, self.cam_w,
                                        self.cam_every, int(force), self._stream()), "bb_render_depth")

    def render_depth(self, force: bool = True) -> torch.Tensor:
        """Depth images [N, 2, H, W] of cam_0/cam_1 at the current state (linear depth, clipped to 1 m)."""
        if not self.cameras:
            raise RuntimeError("cameras are disabled (BallbotVecEnv(..., disable_cameras=False))")
        self._render(force)
        return self.depth

    def step(self, actions: torch.Tensor):
        """One env.step for all envs: returns (obs[N,15], reward[N], terminated[N], truncated[N], info)."""
        if actions.device != self.device or actions.dtype != torch.float32 or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.shape != (self.num_envs, 3):
            raise ValueError(f"actions must have shape ({self.num_envs}, 3), got {tuple(actions.shape)}")
        N.check(N.lib().bb_step(self._h, _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                                _ptr(self.terminal_obs), _ptr(self.pos2d), int(self.auto_reset), self._stream()),
                "bb_step")
        if self.cameras:  # envs whose counter hit the frame interval (incl. auto-resets) re-render
            self._render(force=False)
        if self._reward_error:  # after mj_step, as the reference's reward call (ballbot_env.py:912, 929)
            raise ValueError(self._reward_error)
        terminated = (self.done & N.DONE_TERMINATED) != 0
        info = {"done_flags": self.done, "terminal_observation": self.terminal_obs, "pos2d": self.pos2d,
                "failure": (self.done & N.DONE_FAILURE) != 0}
        reward = self.reward
        if self._host_reward is not None:
            reward = self._plugin_reward(info["failure"])
        return self.obs, reward, terminated, torch.zeros_like(terminated), info

    def step_flags(self, actions: torch.Tensor):
        """env.step without the derived tensors, for the batched trainer's
        rollout: -> (obs[N,15], reward[N], done_flags[N] uint8, BB_DONE_* bits).
        Same launch and buffers as step()."""
        if self._host_reward is not None:
            obs, reward, _, _, info = self.step(actions)
            return obs, reward, info["done_flags"]
        if self._reward_error:
            raise ValueError(self._reward_error)
        if actions.device != self.device or actions.dtype != torch.float32 or not actions.is_contiguous() \
                or actions.shape != (self.num_envs, 3):
            raise ValueError(f"actions must be a contiguous float32 ({self.num_envs}, 3) tensor on {self.device}")
        N.check(N.lib().bb_step(self._h, _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                                _ptr(self.terminal_obs), _ptr(self.pos2d), int(self.auto_reset), self._stream()),
                "bb_step")
        if self.cameras:
            self._render(force=False)
        return self.obs, self.reward, self.done

    def capture_step(self, actions: torch.Tensor) -> "torch.cuda.CUDAGraph":
        """Capture one env.step (routing, fast/full step kernels on the env's two
        streams, depth cameras) reading `actions` as ONE HIP graph; replay() then
        steps every env with whatever `actions` holds (one launch per rollout step)."""
        if actions.shape != (self.num_envs, 3) or actions.dtype != torch.float32 or not actions.is_contiguous():
            raise ValueError("capture_step needs a contiguous float32 [num_envs, 3] action buffer")
        if self._reward_error:
            raise ValueError(self._reward_error)
        graph = torch.cuda.CUDAGraph()
        self.note_graph_capture()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        torch.cuda.synchronize(self.device)
        with torch.cuda.graph(graph, stream=side):
            self._step_launch(actions)
        torch.cuda.synchronize(self.device)
        return graph

    def note_graph_capture(self) -> None:
        """Record that a HIP graph holding this env's handle exists (it lives as long as the env):
        a re-seed that would need a new handle then raises instead of leaving the graph stale."""
        self._graphs += 1

    def _step_launch(self, actions: torch.Tensor) -> None:
        N.check(N.lib().bb_step(self._h, _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                                _ptr(self.terminal_obs), _ptr(self.pos2d), int(self.auto_reset), self._stream()),
                "bb_step")
        if self.cameras:
            self._render(force=False)

    def step_multi(self, actions: torch.Tensor, out: Optional[dict] = None) -> dict:
        """K env.steps of all envs in ONE launch for actions known in advance
        (bb_step_multi; open-loop sequences such as random-action benchmarks):
        actions [K, N, 3] -> {"obs" [K,N,15], "reward" [K,N], "done" [K,N] uint8,
        "terminal_obs" [K,N,15], "pos2d" [K,N,2]}, identical to K step() calls
        (auto-reset, counters and terrain draws included).  `out` (a dict
        returned before, same K) is refilled instead of allocating.  The env's
        obs/reward/done buffers are not updated; cameras are not rendered."""
        if self.cameras:
            raise RuntimeError("step_multi does not render the depth cameras; step() does")
        if self._host_reward is not None:
            raise RuntimeError("step_multi needs a built-in reward (a host plugin runs per step())")
        if self._reward_error:
            raise ValueError(self._reward_error)
        if actions.device != self.device or actions.dtype != torch.float32 or not actions.is_contiguous() \
                or actions.dim() != 3 or actions.shape[1:] != (self.num_envs, 3):
            raise ValueError(f"actions must be a contiguous float32 (K, {self.num_envs}, 3) tensor on {self.device}")
        k = int(actions.shape[0])
        if out is None or out["reward"].shape[0] != k:
            n = self.num_envs
            out = {"obs": torch.empty(k, n, 15, device=self.device), "reward": torch.empty(k, n, device=self.device),
                   "done": torch.empty(k, n, dtype=torch.uint8, device=self.device),
                   "terminal_obs": torch.empty(k, n, 15, device=self.device),
                   "pos2d": torch.empty(k, n, 2, device=self.device)}
        N.check(N.lib().bb_step_multi(self._h, _ptr(actions), k, _ptr(out["obs"]), _ptr(out["reward"]),
                                      _ptr(out["done"]), _ptr(out["terminal_obs"]), _ptr(out["pos2d"]),
                                      int(self.auto_reset), self._stream()), "bb_step_multi")
        return out

    def step_multi_raw(self, actions: torch.Tensor, obs: torch.Tensor, reward: torch.Tensor,
                       done: torch.Tensor, terminal_obs: Optional[torch.Tensor] = None,
                       pos2d: Optional[torch.Tensor] = None) -> None:
        """Launch-only bb_step_multi (benchmarking): caller-owned [K, N, ...] outputs
        (terminal obs / pos2d optional)."""
        N.check(N.lib().bb_step_multi(self._h, _ptr(actions), int(actions.shape[0]), _ptr(obs), _ptr(reward),
                                      _ptr(done), _ptr(terminal_obs), _ptr(pos2d), int(self.auto_reset),
                                      self._stream()), "bb_step_multi")

    def check(self) -> None:
        """Wait for the env's stream and raise if a bb_step_multi relief-pair launch ended on its
        wall-clock budget (bb_check).  The fault is sticky: step(), step_multi() and rollouts raise
        too, without a sync, until a full reset() clears it."""
        N.check(N.lib().bb_check(self._h, self._stream()), "bb_check")

    def run_rollout(self, args) -> None:
        """One whole PPO rollout in one launch (bb_rollout; args: _native.RolloutArgs
        filled by the trainer).  Built-in rewards only; the cameras are not rendered."""
        if self.cameras:
            raise RuntimeError("bb_rollout steps the proprio policy; the camera policy rolls out per step")
        if self._host_reward is not None:
            raise RuntimeError("bb_rollout needs a built-in reward (a host plugin runs per step())")
        if self._reward_error:
            raise ValueError(self._reward_error)
        N.check(N.lib().bb_rollout(self._h, C.byref(args), self._stream()), "bb_rollout")

    def step_async_raw(self, actions: torch.Tensor, full_outputs: bool = False) -> None:
        """Launch-only step (graph capture / benchmarking): no derived tensors;
        full_outputs: also the terminal obs and pos2d buffers."""
        N.check(N.lib().bb_step(self._h, _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                                _ptr(self.terminal_obs) if full_outputs else None,
                                _ptr(self.pos2d) if full_outputs else None, int(self.auto_reset), self._stream()),
                "bb_step")

    def _plugin_reward(self, failure: torch.Tensor) -> torch.Tensor:
        """Reward of a custom plugin, in the reference's float32 order
        (ballbot_env.py:929-937, 1019-1020): plugin(obs) * scale + action penalty
        (the kernel's reward for BB_REWARD_NONE), then + survival bonus unless failed.
        The plugin sees this step's observation (before any auto-reset) and pos2d."""
        f32 = np.float32
        hb = getattr(type(self._host_reward), "has_batched", None)
        if hb is not None and hb():  # device path: one call, no host sync
            st = {k: self.terminal_obs[:, 3 * i:3 * i + 3] for i, k in enumerate(OBS_KEYS)}
            st["pos2d"] = self.pos2d
            v = torch.as_tensor(self._host_reward.batched(st), device=self.device).to(torch.float32).reshape(-1)
            if v.shape[0] != self.num_envs:
                raise ValueError(f"{type(self._host_reward).__name__}.batched returned {v.shape[0]} rewards "
                                 f"for {self.num_envs} envs")
        else:  # compatibility path: BaseReward.__call__(state) per env on the host
            obs = self.terminal_obs.cpu().numpy()
            pos = self.pos2d.cpu().numpy()
            out = np.zeros(self.num_envs, dtype=f32)
            for i in range(self.num_envs):
                state = split_obs(obs[i])
                state["pos2d"] = pos[i]
                out[i] = f32(self._host_reward(state))
            v = torch.from_numpy(out).to(self.device)
        r = v * f32(self._params.reward_scale) + self.reward
        return torch.where(failure, r, r + f32(self._params.survival_bonus))

    # ------------------------------------------------- SB3 VecEnv interface
    def step_async(self, actions) -> None:
        """VecEnv.step_async: remember the actions (torch [N,3] or numpy); step_wait runs the step."""
        self._pending_actions = torch.as_tensor(actions, dtype=torch.float32, device=self.device)

    def step_wait(self):
        """VecEnv.step_wait -> (obs dict of [N,...] tensors, rewards [N], dones [N] bool, infos list).

        dones = terminated (the reference never truncates); done envs were reset
        in the same launch, their last observation is infos[i]["terminal_observation"]
        (SB3's convention).  The per-env info dicts are host objects: the batched
        trainer reads the tensors of step() instead."""
        if self._pending_actions is None:
            raise RuntimeError("step_wait() without step_async()")
        obs, reward, term, trunc, info = self.step(self._pending_actions)
        self._pending_actions = None
        done = term | trunc
        d_h = done.cpu().numpy()
        fail = info["failure"].cpu().numpy()
        p2 = info["pos2d"].cpu().numpy()
        tob = info["terminal_observation"].cpu().numpy()
        infos = []
        for i in range(self.num_envs):
            inf = {"TimeLimit.truncated": False, "failure": bool(fail[i]), "success": False, "pos2d": p2[i]}
            if d_h[i]:
                inf["terminal_observation"] = split_obs(tob[i])
            infos.append(inf)
        return self.obs_dict(obs), reward, done, infos

    def seed(self, seed: Optional[int] = None):
        """VecEnv.seed (SB3 2.x): env i re-seeds to np_random(seed + i) at the next
        reset() -- the terrain generator, as reset(seed=seed+i) replaces the
        reference env's _np_random (ballbot_env.py:596) -- and the action space is
        seeded.  seed None: a random base, as SB3 draws one.  -> the seeds."""
        if seed is None:
            seed = int(np.random.randint(0, np.iinfo(np.uint32).max, dtype=np.uint32))
        self._pending_seeds = [int(seed) + i for i in range(self.num_envs)]
        self.action_space.seed(seed)
        return list(self._pending_seeds)

    def load_terrain(self, slot: int, seed: Optional[int]) -> None:
        """Generate the terrain of `seed` (the registered plugin, or the GPU perlin
        generator) into bank slot `slot` (terrain_slots mode; ballbot_env.py:501-513)."""
        from .config import _gen_chunk, perlin_cfg

        L = N.lib()
        size_z = self.terrain_plan.size_z
        if self._gpu_perlin() and seed is not None:
            sd = np.array([int(seed)], np.int32)
            N.check(L.bb_generate_perlin(self._h, int(slot), 1, sd.ctypes.data_as(C.POINTER(C.c_int32)),
                                         C.byref(perlin_cfg(self.terrain_config)), float(size_z)),
                    "bb_generate_perlin")
        else:
            arr = np.ascontiguousarray(_gen_chunk(self.terrain_config, [seed], N.HF_N)[0], dtype=np.float32)
            N.check(L.bb_set_hfield(self._h, int(slot), arr.ctypes.data_as(C.POINTER(C.c_float)), float(size_z)),
                    "bb_set_hfield")
        self.terrain_seeds[int(slot)] = seed if seed is not None else -1

    def terrain_rng(self):
        """(uint64[N][5] device generators in pcg64_words form (None without generators), int32[N] terrain seed of
        each env's last device draw, -1 before the first)."""
        gen = self.terrain_plan.stream_seeds is not None
        w = np.zeros((self.num_envs, 5), np.uint64) if gen else None
        s = np.zeros(self.num_envs, np.int32)
        N.check(N.lib().bb_get_terrain_rng(self._h, None if w is None else w.ctypes.data_as(C.POINTER(C.c_uint64)),
                                           s.ctypes.data_as(C.POINTER(C.c_int32))), "bb_get_terrain_rng")
        return w, s

    def get_attr(self, name: str, indices=None):
        n = self.num_envs if indices is None else len(list(indices))
        return [getattr(self, name)] * n

    def set_attr(self, name: str, value, indices=None) -> None:
        setattr(self, name, value)

    def env_method(self, name: str, *args, indices=None, **kwargs):
        n = self.num_envs if indices is None else len(list(indices))
        return [getattr(self, name)(*args, **kwargs)] * n

    def env_is_wrapped(self, wrapper_class, indices=None):
        n = self.num_envs if indices is None else len(list(indices))
        return [False] * n

    def obs_dict(self, obs: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        o = self.obs if obs is None else obs
        d = {k: o[:, 3 * i:3 * i + 3] for i, k in enumerate(OBS_KEYS)}
        if self.cameras:  # the reference's camera keys (ballbot_env.py:812-826), channels-first
            d["rgbd_0"] = self.depth[:, 0:1]
            d["rgbd_1"] = self.depth[:, 1:2]
            d["relative_image_timestamp"] = self.rel_ts.unsqueeze(1)
        return dict(sorted(d.items()))

    # ------------------------------------------------------------ parity/state
    def get_state(self):
        n = self.num_envs
        q, v, w = np.zeros((n, N.NQ)), np.zeros((n, N.NV)), np.zeros((n, N.NV))
        s = np.zeros(n, dtype=np.int32)
        dp = C.POINTER(C.c_double)
        N.check(N.lib().bb_get_state(self._h, q.ctypes.data_as(dp), v.ctypes.data_as(dp), w.ctypes.data_as(dp),
                                     s.ctypes.data_as(C.POINTER(C.c_int32))), "bb_get_state")
        return q, v, w, s

    def set_state(self, qpos, qvel, warm=None, steps=None):
        n = self.num_envs
        q = np.ascontiguousarray(np.broadcast_to(qpos, (n, N.NQ)), dtype=np.float64)
        v = np.ascontiguousarray(np.broadcast_to(qvel, (n, N.NV)), dtype=np.float64)
        w = np.zeros((n, N.NV)) if warm is None else np.ascontiguousarray(np.broadcast_to(warm, (n, N.NV)),
                                                                           dtype=np.float64)
        s = np.zeros(n, np.int32) if steps is None else np.ascontiguousarray(np.broadcast_to(steps, (n,)),
                                                                              dtype=np.int32)
        dp = C.POINTER(C.c_double)
        N.check(N.lib().bb_set_state(self._h, q.ctypes.data_as(dp), v.ctypes.data_as(dp), w.ctypes.data_as(dp),
                                     s.ctypes.data_as(C.POINTER(C.c_int32))), "bb_set_state")

    def forward(self, ctrl):
        """mj_forward at the current state (diagnostic): returns qacc [N,15] and contact
        counts [N,2] = (ball-hfield, base-tree geoms)."""
        n = self.num_envs
        c = np.ascontiguousarray(np.broadcast_to(ctrl, (n, 3)), dtype=np.float64)
        qacc = np.zeros((n, N.NV))
        ncon = np.zeros((n, 2), np.int32)
        dp = C.POINTER(C.c_double)
        N.check(N.lib().bb_forward(self._h, c.ctypes.data_as(dp), qacc.ctypes.data_as(dp),
                                   ncon.ctypes.data_as(C.POINTER(C.c_int32))), "bb_forward")
        return qacc, ncon

    def stats(self) -> Dict[str, int]:
        out = (C.c_int64 * N.NSTATS)()
        N.check(N.lib().bb_get_stats(self._h, out, N.NSTATS), "bb_get_stats")
        return {"resets": out[0], "diverged": out[1], "overflow": out[2], "slow_path": out[3],
                "solver_iters": out[4], "stream_wraps": out[5], "spill": out[6], "pair_budget": out[7]}

    def pair_counters(self) -> Dict[str, int]:
        """Diagnostics of the last relief-pair launch of step_multi (bb_pair_counters; waits for the device)."""
        keys = ("busy_fast", "busy_full", "idle_fast", "idle_full", "active_fast", "active_full", "claims_fast",
                "claims_full", "steps_fast", "steps_full", "handovers", "life_cycles_fast", "life_cycles_full",
                "life_wall_fast", "life_wall_full", "heavy", "ring_len", "ring_pushes_min_fast", "ring_pushes_min_full")
        out = (C.c_int64 * len(keys))()
        N.check(N.lib().bb_pair_counters(self._h, out, len(keys)), "bb_pair_counters")
        return dict(zip(keys, out))

    def pair_env_times(self):
        """Per env, the last relief-pair launch: (shader cycles its steps took, wall tick of its last step)."""
        out = np.zeros((2, self.num_envs), np.uint64)
        N.check(N.lib().bb_pair_env_times(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64))), "bb_pair_env_times")
        return out[0], out[1]

    def env_terrain(self):
        """(bank slot of every env's current terrain, stream draws each env made) as int32[N] arrays."""
        t = np.zeros(self.num_envs, np.int32)
        k = np.zeros(self.num_envs, np.int32)
        ip = C.POINTER(C.c_int32)
        N.check(N.lib().bb_get_env_terrain(self._h, t.ctypes.data_as(ip), k.ctypes.data_as(ip)), "bb_get_env_terrain")
        return t, k

    def assign_terrain(self, ids) -> None:
        """Pin env i to bank slot ids[i] for its later resets (-1 unpins: back to its stream)."""
        t = torch.as_tensor(np.asarray(ids, np.int32)).to(self.device)
        N.check(N.lib().bb_assign_terrain(self._h, _ptr(t), self._stream()), "bb_assign_terrain")
        torch.cuda.current_stream(self.device).synchronize()

    def hfield(self, terrain_id: int) -> np.ndarray:
        """Terrain bank slot `terrain_id` as float32[293*293] (host copy)."""
        out = np.empty(N.HF_N * N.HF_N, np.float32)
        N.check(N.lib().bb_get_hfield(self._h, int(terrain_id), out.ctypes.data_as(C.POINTER(C.c_float))),
                "bb_get_hfield")
        return out

    def time_kernel(self, max_launches: int) -> None:
        """Time the next `max_launches` fast step kernels with HIP events (bench.py)."""
        N.check(N.lib().bb_time_kernel(self._h, int(max_launches)), "bb_time_kernel")

    def kernel_ms(self):
        """(average fast-step-kernel duration in ms, launches timed) since time_kernel()."""
        ms, k = C.c_double(), C.c_int32()
        N.check(N.lib().bb_kernel_ms(self._h, C.byref(ms), C.byref(k)), "bb_kernel_ms")
        return ms.value, k.value

    def kernel_times(self):
        """Average ms of the fast kernel, the predicted full kernel (route 0, side stream) and
        the hand-over full kernel over the steps timed since time_kernel(); and the count."""
        t, k = (C.c_double * 3)(), C.c_int32()
        N.check(N.lib().bb_kernel_times(self._h, t, C.byref(k)), "bb_kernel_times")
        return {"fast": t[0], "predicted_full": t[1], "handover_full": t[2]}, k.value

    def launch_config(self) -> Dict[str, int]:
        out = (C.c_int32 * 5)()
        N.check(N.lib().bb_get_config(self._h, out), "bb_get_config")
        return {"num_envs": out[0], "envs_per_wave": out[1], "fp64": out[2], "lds_bytes_per_workgroup": out[3],
                "lanes_per_env": out[4]}

    def offsets(self) -> np.ndarray:
        o = np.zeros(self.n_terrains, np.float32)
        N.check(N.lib().bb_get_offsets(self._h, o.ctypes.data_as(C.POINTER(C.c_float))), "bb_get_offsets")
        return o

    def close(self):
        if getattr(self, "_h", None):
            N.lib().bb_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def split_obs(obs15) -> Dict[str, Any]:
    return {k: obs15[3 * i:3 * i + 3] for i, k in enumerate(OBS_KEYS)}
