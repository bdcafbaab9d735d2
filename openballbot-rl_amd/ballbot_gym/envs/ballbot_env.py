"""BBotSimulation: the reference's single-env Gym surface over the batched HIP step.

Drop-in for `ballbot_gym.envs.ballbot_env.BBotSimulation` (reference
ballbot_env.py:60-1036) as `make("ballbot-v0.1", ...)` builds it: same
constructor keywords (:157-178), `reset(seed=None, goal="random") -> (obs,
info)` (:567), `step(a: float32[3]) -> (obs, reward, terminated, truncated,
info)` (:854), `action_space` / `observation_space` (:235-256), `close()`.
One env = a BallbotVecEnv of one env on the GPU with auto-reset off: the
physics, observation, reward and termination run in the same HIP kernels as
the batched path.  Observations are dicts of float32 numpy arrays (the
reference's keys; camera keys when cameras are on), the reward a Python float
(the float32 value: the reference's tests check isinstance(reward, float)).

Terrain seeds as the reference draws them (:378-384, :505-510, :596-599,
:658-661): eval_env=[True, s] fixes _np_random = np_random(s) at
construction; reset(seed=s) with s not None replaces it by np_random(s)
(gymnasium's Env.reset, :596), in eval mode too; a reset with no generator yet
seeds one from OS entropy (:597-599).  Every reset draws r_seed =
integers(0, 10000) from it (unless the terrain config fixes a seed), and a
non-eval env's first reset then draws the log-dir permutation (:655-661).  The
host runs that generator and generates the drawn terrain into a small ring of
bank slots (the GPU perlin generator, or the registered plugin), as the
reference regenerates the heightfield at every reset (:501-513).

Not provided: the MuJoCo viewer (GUI), RGB video rendering (`render()`) and
the per-episode log files (_save_logs) -- outside the hot path.
"""
from __future__ import annotations

import string
from collections import OrderedDict
from typing import Any, Dict, Optional

import numpy as np

from .. import spaces
from .config import np_random

DT = 0.002  # ballbot.xml:3 (opt.timestep)
RING_SLOTS = 4  # bank slots of the single env: the terrains of its latest draws


class BBotSimulation:
    metadata = {"render_modes": ["rgb_array"], "render_fps": 30}

    def __init__(self, xml_path=None, GUI=False, im_shape=None, disable_cameras=False, depth_only=True,
                 log_options=None, max_ep_steps=None, terrain_type: str = "perlin", eval_env=(False, None),
                 reward_config=None, terrain_config=None, env_config=None, render_mode: Optional[str] = None,
                 viewer_title: Optional[str] = None, device: str = "cuda:0", precision: str = "fp64",
                 n_terrains: Optional[int] = None, reward_compat: str = "reference"):
        if render_mode is not None and render_mode not in self.metadata["render_modes"]:
            raise ValueError(f"Invalid render_mode: {render_mode}. Supported modes: {self.metadata['render_modes']}")
        if GUI:
            raise ValueError("GUI (the MuJoCo passive viewer) is not available in the MI355X build")
        im_shape = im_shape or {"h": 64, "w": 64}
        self.terrain_config = terrain_config if terrain_config is not None else {"type": terrain_type, "config": {}}
        self.terrain_type = self.terrain_config.get("type", terrain_type)
        self.reward_config = reward_config or {"type": "directional", "config": {"target_direction": [0.0, 1.0]}}
        env_config = dict(env_config or {})
        cam = dict(env_config.get("camera", {}) or {})
        depth = cam.get("disable_rgb", depth_only) if cam else depth_only
        if not disable_cameras and not depth:
            raise ValueError("only depth cameras are rendered (depth_only / camera.disable_rgb must be true)")
        cam.setdefault("height", im_shape["h"])
        cam.setdefault("width", im_shape["w"])
        cam["disable_rgb"] = True
        env_config["camera"] = cam
        self._env_config = env_config
        self.max_ep_steps = int((env_config.get("env", {}) or {}).get(
            "max_ep_steps", max_ep_steps if max_ep_steps is not None else 4000))
        self.disable_cameras = bool(disable_cameras)
        self.xml_path = xml_path
        self.log_options = log_options or {"cams": False, "reward_terms": False}
        self.render_mode = render_mode if render_mode is not None else "rgb_array"
        self.viewer_title = viewer_title
        self.passive_viewer = None
        self.log_dir = None
        self.action_space = spaces.action_space()
        self.observation_space = spaces.observation_space({"h": cam["height"], "w": cam["width"]}, 1,
                                                          self.disable_cameras)
        self.eval_env = bool(eval_env[0])
        self.step_counter = 0
        self.num_episodes = -1
        self.last_r_seed = None
        self._log_drawn = False  # the non-eval log-dir permutation (first reset only, ballbot_env.py:655-661)
        # eval mode: _np_random fixed now (ballbot_env.py:378-384); else seeded by the first reset
        self._np_random = np_random(eval_env[1]) if self.eval_env else None
        # a ring of bank slots holding the terrains of the latest draws (n_terrains slots, default 4)
        from .vec_env import BallbotVecEnv

        self._ring = max(1, int(n_terrains or RING_SLOTS))
        self._slot_of: "OrderedDict[int, int]" = OrderedDict()
        self._env = BallbotVecEnv(1, device=device, reward_config=self.reward_config,
                                  terrain_config=self.terrain_config, env_config=self._env_config,
                                  max_ep_steps=max_ep_steps, precision=precision, auto_reset=False,
                                  disable_cameras=self.disable_cameras, terrain_slots=self._ring,
                                  reward_compat=reward_compat)

    @property
    def opt_timestep(self) -> float:
        return DT

    @property
    def np_random(self) -> np.random.Generator:
        """gymnasium's Env.np_random: the terrain generator (seeded from OS entropy if unset)."""
        if self._np_random is None:
            self._np_random = np_random(None)
        return self._np_random

    # ------------------------------------------------------------------ setup
    def _slot(self, r_seed) -> int:
        """Bank slot holding the terrain of r_seed, generated into the least
        recently used ring slot if it is not resident (ballbot_env.py:501-513)."""
        from .config import terrain_is_seedless

        tc = self.terrain_config
        key = -1 if (tc.get("type", "flat") == "flat" or terrain_is_seedless(tc)) else int(r_seed)
        if key in self._slot_of:
            self._slot_of.move_to_end(key)
            return self._slot_of[key]
        if len(self._slot_of) < self._ring:
            slot = len(self._slot_of)
        else:
            _, slot = self._slot_of.popitem(last=False)
        self._env.load_terrain(slot, None if key == -1 and tc.get("type", "flat") == "flat" else int(r_seed))
        self._slot_of[key] = slot
        return slot

    # -------------------------------------------------------------------- api
    def reset(self, seed=None, goal: str = "random", **kwargs):
        """ballbot_env.py:567-671: (re)seed the generator, draw the terrain seed,
        init height offset, zero state -> (obs, info)."""
        from .config import TERRAIN_SEED_HIGH

        if seed is not None:  # gymnasium Env.reset(seed) replaces _np_random (ballbot_env.py:596)
            self._np_random = np_random(seed)
        gen = self.np_random
        cfg_seed = (self.terrain_config.get("config", {}) or {}).get("seed")
        r_seed = int(gen.integers(0, TERRAIN_SEED_HIGH)) if cfg_seed is None else int(cfg_seed)
        self.last_r_seed = r_seed
        if not self.eval_env and not self._log_drawn:  # the /tmp/log_<12 chars> name (ballbot_env.py:655-661)
            gen.permutation(list(string.ascii_letters + string.digits))
            self._log_drawn = True
        self._env.assign_terrain(np.array([self._slot(r_seed)], np.int32))
        self._env.reset()
        self.num_episodes += 1
        self.step_counter = 0
        obs = self._obs()
        return obs, self._info(np.zeros(2, np.float32), False)

    def step(self, action):
        """ballbot_env.py:854-1036 for this env: (obs, reward, terminated, truncated, info)."""
        import torch

        a = np.asarray(action, dtype=np.float32).reshape(1, 3)
        obs, rew, term, trunc, info = self._env.step(torch.from_numpy(a).to(self._env.device))
        self.step_counter += 1
        fl = int(info["done_flags"][0].item())
        return (self._obs(), float(rew[0].item()), bool(fl & 1), False,
                self._info(info["pos2d"][0].cpu().numpy().astype(np.float32), bool(fl & 2)))

    def close(self):
        if self._env is not None:
            self._env.close()
            self._env = None

    # ---------------------------------------------------------------- helpers
    def _obs(self) -> Dict[str, Any]:
        d = self._env.obs_dict()
        out = {k: d[k][0].detach().cpu().numpy().astype(np.float32) for k in
               ("orientation", "angular_vel", "vel", "motor_state", "actions")}
        if not self.disable_cameras:
            for k in ("rgbd_0", "rgbd_1", "relative_image_timestamp"):
                out[k] = d[k][0].detach().cpu().numpy().astype(np.float32)
        return out

    def _info(self, pos2d, failure: bool) -> Dict[str, Any]:
        """_get_info (ballbot_env.py:831-852) plus the step's failure flag (:1009-1011)."""
        return {"success": False, "failure": failure, "step_counter": self.step_counter, "pos2d": pos2d}

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
