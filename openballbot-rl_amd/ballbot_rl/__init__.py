"""ballbot_rl (MI355X-native): the trainer side of the hot path.

The reference trains with stable-baselines3 PPO over a SubprocVecEnv of CPU
MuJoCo envs (ballbot_rl/training/train.py).  Here the rollout runs on the GPU
against BallbotVecEnv (thousands of envs per launch), GAE runs as a HIP kernel
(bb_gae), and the PPO update follows SB3 2.6.0's semantics on device tensors.
"""
__version__ = "0.1.0"
