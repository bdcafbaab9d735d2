"""Policy evaluation (reference ballbot_rl/evaluation)."""
from ballbot_rl.evaluation.evaluate import evaluate_policy

__all__ = ["evaluate_policy"]
