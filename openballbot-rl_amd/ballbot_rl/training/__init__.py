"""Training: batched PPO over the GPU env (reference ballbot_rl/training)."""
from ballbot_rl.training.logger import CSVLogger, read_progress
from ballbot_rl.training.schedules import lr_schedule

__all__ = ["CSVLogger", "read_progress", "lr_schedule"]
