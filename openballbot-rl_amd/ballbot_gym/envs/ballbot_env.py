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
construction; otherwise the generator is np_random(seed) of the FIRST reset,
and that first reset also draws the log-dir permutation after its terrain
draw.  Every later reset draws the next value of integers(0, 10000).

Not provided: the MuJoCo viewer (GUI), RGB video rendering (`render()`) and
the per-episode log files (_save_logs) -- outside the hot path.
"""
from __future__ import annotations

import string
from typing import Any, Dict, Optional

import numpy as np

from .. import spaces
from .config import np_random

DT = 0.002  # ballbot.xml:3 (opt.timestep)


class BBotSimulation:
    metadata = {"render_modes": ["rgb_array"], "render_fps": 30}

    def __init__(self, xml_path=None, GUI=False, im_shape=None, disable_cameras=False, depth_only=True,
                 log_options=None, max_ep_steps=None, terrain_type: str = "perlin", eval_env=(False, None),
                 reward_config=None, terrain_config=None, env_config=None, render_mode: Optional[str] = None,
                 viewer_title: Optional[str] = None, device: str = "cuda:0", precision: str = "fp64",
                 n_terrains: Optional[int] = None):
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
        self._max_ep_steps_arg = max_ep_steps
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
        self._device, self._precision, self._n_terrains = device, precision, n_terrains
        self.eval_env = bool(eval_env[0])
        self._eval_seed = eval_env[1]
        self._env = None
        self.step_counter = 0
        self.num_episodes = -1
        self.last_r_seed = None
        if self.eval_env:  # _np_random fixed now (ballbot_env.py:378-384); the first reset draws from it
            self._build(np_random(self._eval_seed), first_permutation=False)

    @property
    def opt_timestep(self) -> float:
        return DT

    # ------------------------------------------------------------------ setup
    def _build(self, gen: np.random.Generator, first_permutation: bool) -> None:
        """The backing one-env BallbotVecEnv, with this env's terrain stream."""
        from .config import FULL_BANK_DRAWS_PER_ENV, NUMPY_BANK_DRAWS, TERRAIN_SEED_HIGH
        from .vec_env import BallbotVecEnv

        k = self._n_terrains or (FULL_BANK_DRAWS_PER_ENV if self.terrain_type == "perlin" else NUMPY_BANK_DRAWS)
        draws = [int(gen.integers(0, TERRAIN_SEED_HIGH))]
        if first_permutation:  # the log-dir name of a non-eval env's first reset (ballbot_env.py:658-661)
            gen.permutation(list(string.ascii_letters + string.digits))
        draws += [int(x) for x in gen.integers(0, TERRAIN_SEED_HIGH, size=k - 1)]
        self._draws = draws
        self._env = BallbotVecEnv(1, device=self._device, reward_config=self.reward_config,
                                  terrain_config=self.terrain_config, env_config=self._env_config,
                                  max_ep_steps=self._max_ep_steps_arg, precision=self._precision,
                                  n_terrains=k,  # the bank holds the distinct seeds of these draws
                                  auto_reset=False, disable_cameras=self.disable_cameras,
                                  terrain_draws=draws)
        self._fresh = True  # constructed = reset once (draw 0)

    # -------------------------------------------------------------------- api
    def reset(self, seed=None, goal: str = "random", **kwargs):
        """ballbot_env.py:567-671: next terrain draw, init height offset, zero state -> (obs, info)."""
        if self._env is None:  # non-eval: _np_random = np_random(seed of the first reset)
            self._build(np_random(seed), first_permutation=True)
        if self._fresh:
            self._fresh = False
        else:
            self._env.reset()
        self.num_episodes += 1
        self.step_counter = 0
        cfg_seed = (self.terrain_config.get("config", {}) or {}).get("seed")
        self.last_r_seed = cfg_seed if cfg_seed is not None else self._draws[self.num_episodes % len(self._draws)]
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
