"""Actor-critic policy with the reference's feature extractor (ballbot_rl/policies/mlp_policy.py:7-163).

The reference builds stable-baselines3's MultiInputPolicy with
* features_extractor = Extractor: one branch per observation key, iterated in
  the Dict space's (sorted) key order; proprio keys are flattened, `rgbd_*`
  keys go through a 2-conv CNN (32 filters, k3 s2 p1, BatchNorm, LeakyReLU,
  Linear to 20, BatchNorm1d, Tanh) or a frozen encoder; the branch outputs are
  concatenated (mlp_policy.py:143-163) and shared by actor and critic;
* net_arch pi = vf = [hidden_sz]*4 with LeakyReLU (train.py:39-52);
* SB3 ActorCriticPolicy defaults: DiagGaussian head with a state-independent
  log_std initialised to 0, orthogonal init with gains sqrt(2) (extractor, MLP
  trunks), 0.01 (action net), 1 (value net) and zero biases.
SB3 itself is not installed; this restates its published semantics.

Observations may be a dict of tensors or the packed [N, 15] proprio tensor that
BallbotVecEnv returns (already in sorted-key order, so flattening and
concatenating the dict is the identity on it).
"""
from __future__ import annotations

import copy
import math
import os
from collections import OrderedDict
from typing import Dict, Optional, Sequence, Tuple, Union

import torch
from torch import nn

PROPRIO_KEYS = ("actions", "angular_vel", "motor_state", "orientation", "vel")
Obs = Union[torch.Tensor, Dict[str, torch.Tensor]]


def obs_spaces(cameras: bool = False, channels: int = 1, height: int = 64, width: int = 64) -> "OrderedDict":
    """Observation key -> shape, in gymnasium Dict (sorted) order (ballbot_env.py:701-767)."""
    sp = {k: (3,) for k in PROPRIO_KEYS}
    if cameras:
        sp["relative_image_timestamp"] = (1,)
        sp["rgbd_0"] = (channels, height, width)
        sp["rgbd_1"] = (channels, height, width)
    return OrderedDict(sorted(sp.items()))


def depth_cnn(C: int, H: int, W: int, out_sz: int = 20) -> nn.Sequential:
    """The reference's per-camera CNN (mlp_policy.py:25-46)."""
    F1 = F2 = 32
    return nn.Sequential(
        nn.Conv2d(C, F1, kernel_size=3, stride=2, padding=1), nn.BatchNorm2d(F1), nn.LeakyReLU(),
        nn.Conv2d(F1, F2, kernel_size=3, stride=2, padding=1), nn.BatchNorm2d(F2), nn.LeakyReLU(),
        nn.Flatten(), nn.Linear(F2 * H // 4 * W // 4, out_sz), nn.BatchNorm1d(out_sz), nn.Tanh())


class Extractor(nn.Module):
    """Per-key extractors concatenated in key order (mlp_policy.py:7-163).

    `frozen_encoder`: an nn.Module (e.g. loaded from a safetensors state dict by
    the caller) used, frozen, for every rgbd key instead of a trainable CNN.
    The reference's torch.load of a pickled module is deliberately not offered."""

    def __init__(self, observation_space: Dict[str, Sequence[int]], frozen_encoder: Optional[nn.Module] = None):
        super().__init__()
        ex = {}
        total = 0
        for key, shape in observation_space.items():
            if "rgbd_" in key:
                if frozen_encoder is None:
                    C, H, W = shape
                    ex[key] = depth_cnn(C, H, W)
                    total += 20
                else:  # one copy per camera key, as the reference loads it once per key (mlp_policy.py:51-54)
                    enc = copy.deepcopy(frozen_encoder)
                    ex[key] = enc
                    total += [m for m in enc.modules() if isinstance(m, nn.Linear)][-1].out_features
                    for p in enc.parameters():
                        p.requires_grad = False
            else:
                ex[key] = nn.Flatten()
                total += int(shape[0])
        self.extractors = nn.ModuleDict(ex)
        self.keys = list(observation_space.keys())
        self.features_dim = total
        self._proprio_only = all(k in PROPRIO_KEYS for k in self.keys)
        # frozen encoders of the reference's layout run as bb_depth_encoder on the GPU
        self._frozen_keys = set()
        if frozen_encoder is not None:
            from ballbot_rl.encoders.models import fusable_encoder

            self._frozen_keys = {k for k in self.keys if "rgbd_" in k and fusable_encoder(ex[k])}

    def forward(self, observations: Obs) -> torch.Tensor:
        if isinstance(observations, torch.Tensor):
            if not self._proprio_only:
                raise ValueError("a packed observation tensor only carries the proprio keys")
            return observations.reshape(observations.shape[0], -1)
        return torch.cat([self._extract(k, observations[k]) for k in self.keys], dim=1)

    def _extract(self, key: str, x: torch.Tensor) -> torch.Tensor:
        # the fused encoder has no autograd graph: an encoder unfrozen after construction
        # (fine-tuning) goes through its torch modules so its gradients are kept
        trainable = torch.is_grad_enabled() and any(p.requires_grad for p in self.extractors[key].parameters())
        if (key in self._frozen_keys and x.is_cuda and not trainable
                and os.environ.get("BB_FUSED_ENCODER", "1") != "0"):
            from ballbot_rl.encoders.models import fused_encoder_forward

            return fused_encoder_forward(self.extractors[key], x)
        return self.extractors[key](x)


class _SplitKLinearFn(torch.autograd.Function):
    """y = x W' + b with the weight gradient split along the batch (split-K).

    For PPO minibatches (B = 8192 rows, 128 features) hipBLASLt computes
    dW = dy' x as one 128x128 GEMM with K = 8192 on 16 workgroups (~48 us,
    profiles/r01 PPO trace); S batched slices of K/S rows plus a sum fill the
    chip.  Same math, fp32, only the summation order changes."""

    @staticmethod
    def forward(ctx, x, w, b, splits):
        ctx.save_for_backward(x, w)
        ctx.splits = splits
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        S = ctx.splits
        B = x.shape[0]
        gx = gy @ w if ctx.needs_input_grad[0] else None
        gw = torch.bmm(gy.reshape(S, B // S, -1).transpose(1, 2), x.reshape(S, B // S, -1)).sum(0)
        gb = gy.sum(0)
        return gx, gw, gb, None


class SplitKLinear(nn.Linear):
    """nn.Linear (same parameters and state dict) whose large-batch GPU backward
    uses the split-K weight gradient: K slices of ROWS rows each, so a 128x128
    dW tile grid has B / ROWS workgroups (128 at B = 8192) instead of 16."""

    ROWS = int(os.environ.get("BB_SPLITK_ROWS", "64"))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0] if x.dim() == 2 else 0
        S = B // self.ROWS if self.ROWS > 0 else 0
        if x.is_cuda and B >= 2048 and S >= 2 and B % S == 0 and torch.is_grad_enabled():
            return _SplitKLinearFn.apply(x, self.weight, self.bias, S)
        return super().forward(x)


def _mlp(sizes: Sequence[int], in_dim: int, act) -> Tuple[nn.Sequential, int]:
    layers = []
    for h in sizes:
        layers += [SplitKLinear(in_dim, h), act()]
        in_dim = h
    return nn.Sequential(*layers), in_dim


class ActorCriticPolicy(nn.Module):
    """SB3 MultiInputPolicy as configured by the reference (train.py:39-56)."""

    LOG_2PI = math.log(2.0 * math.pi)

    def __init__(self, observation_space: Dict[str, Sequence[int]], action_dim: int = 3,
                 net_arch: Optional[Dict[str, Sequence[int]]] = None, activation_fn=nn.LeakyReLU,
                 frozen_encoder: Optional[nn.Module] = None, log_std_init: float = 0.0, ortho_init: bool = True):
        super().__init__()
        net_arch = net_arch or {"pi": [128] * 4, "vf": [128] * 4}
        self.features_extractor = Extractor(observation_space, frozen_encoder)
        fd = self.features_extractor.features_dim
        self.policy_net, pi_dim = _mlp(net_arch["pi"], fd, activation_fn)
        self.value_net_trunk, vf_dim = _mlp(net_arch["vf"], fd, activation_fn)
        self.action_net = SplitKLinear(pi_dim, action_dim)
        self.value_net = SplitKLinear(vf_dim, 1)
        self.log_std = nn.Parameter(torch.full((action_dim,), float(log_std_init)))
        if ortho_init:
            for mod, gain in ((self.features_extractor, math.sqrt(2)), (self.policy_net, math.sqrt(2)),
                              (self.value_net_trunk, math.sqrt(2)), (self.action_net, 0.01), (self.value_net, 1.0)):
                for m in mod.modules():
                    if isinstance(m, (nn.Linear, nn.Conv2d)) and any(p.requires_grad for p in m.parameters()):
                        nn.init.orthogonal_(m.weight, gain=gain)
                        if m.bias is not None:
                            m.bias.data.fill_(0.0)

    # -- distribution pieces (SB3 DiagGaussianDistribution) --
    def _heads(self, obs: Obs):
        f = self.features_extractor(obs)
        return self.action_net(self.policy_net(f)), self.value_net(self.value_net_trunk(f)).squeeze(-1)

    def log_prob(self, mean: torch.Tensor, actions: torch.Tensor) -> torch.Tensor:
        ls = self.log_std
        z = (actions - mean) * torch.exp(-ls)
        return (-0.5 * z * z - ls - 0.5 * self.LOG_2PI).sum(-1)

    def entropy(self, n: int) -> torch.Tensor:
        return (0.5 + 0.5 * self.LOG_2PI + self.log_std).sum().expand(n)

    def forward(self, obs: Obs, deterministic: bool = False, generator: Optional[torch.Generator] = None,
                noise: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """-> (actions, values, log_prob), actions unclipped (SB3 clips before env.step).
        `noise`: standard-normal draws to use instead of sampling (graph replays)."""
        mean, values = self._heads(obs)
        if deterministic:
            actions = mean
        else:
            eps = noise if noise is not None else torch.randn(mean.shape, generator=generator, device=mean.device,
                                                              dtype=mean.dtype)
            actions = mean + eps * torch.exp(self.log_std)
        return actions, values, self.log_prob(mean, actions)

    def evaluate_actions(self, obs: Obs, actions: torch.Tensor):
        """-> (values, log_prob, entropy) for the PPO loss."""
        mean, values = self._heads(obs)
        return values, self.log_prob(mean, actions), self.entropy(actions.shape[0])

    def predict_values(self, obs: Obs) -> torch.Tensor:
        f = self.features_extractor(obs)
        return self.value_net(self.value_net_trunk(f)).squeeze(-1)

    @torch.no_grad()
    def predict(self, obs: Obs, deterministic: bool = True) -> torch.Tensor:
        """Clipped actions in [-1, 1] (SB3 BasePolicy.predict on a Box(-1, 1) action space)."""
        a, _, _ = self.forward(obs, deterministic=deterministic)
        return a.clamp(-1.0, 1.0)
