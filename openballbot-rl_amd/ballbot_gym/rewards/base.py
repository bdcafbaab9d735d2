"""Reward plugin ABI (reference ballbot_gym/rewards/base.py:7-20)."""
from abc import ABC, abstractmethod
from typing import Dict


class BaseReward(ABC):
    """A reward plugin maps one env's observation/state dict to a float."""

    @abstractmethod
    def __call__(self, state: Dict) -> float:
        ...
