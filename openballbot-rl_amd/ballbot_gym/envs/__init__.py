"""Batched (GPU) and single-env views of the ballbot hot path."""
from ballbot_gym.envs.vec_env import BallbotVecEnv, OBS_KEYS, split_obs

__all__ = ["BallbotVecEnv", "OBS_KEYS", "split_obs"]
