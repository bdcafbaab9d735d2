"""Batched (GPU) and single-env views of the ballbot hot path."""
from ballbot_gym.envs.vec_env import BallbotVecEnv, OBS_KEYS, split_obs
from ballbot_gym.envs.ballbot_env import BBotSimulation

__all__ = ["BallbotVecEnv", "BBotSimulation", "OBS_KEYS", "split_obs"]
