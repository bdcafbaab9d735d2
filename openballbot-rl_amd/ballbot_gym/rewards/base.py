"""Reward plugin ABI (reference ballbot_gym/rewards/base.py:7-20).

`__call__(state) -> float` is the reference's per-env ABI.  The batched env
adds an optional device form (SURVEY.md §8 B2's documented extension): a
plugin that overrides `batched(state)` receives the state of all N envs as a
dict of torch tensors on the GPU -- "actions", "angular_vel", "motor_state",
"orientation", "vel" [N, 3] and "pos2d" [N, 2] -- and returns the N rewards
as a tensor, with no host round trip.  Plugins that do not override it are
called once per env on the host (the compatibility path).
"""
from abc import ABC, abstractmethod
from typing import Dict


class BaseReward(ABC):
    """A reward plugin maps one env's observation/state dict to a float."""

    @abstractmethod
    def __call__(self, state: Dict) -> float:
        ...

    def batched(self, state: Dict):
        """Rewards of every env from a dict of [N, ...] device tensors -> tensor [N].
        Not implemented by default: the env then calls __call__ per env."""
        raise NotImplementedError

    @classmethod
    def has_batched(cls) -> bool:
        return cls.batched is not BaseReward.batched
