"""SB3 PPO.train's optimiser step as two HIP launches (bb_adamw_clip).

SB3 2.6.0 PPO.train, after loss.backward(), runs
    th.nn.utils.clip_grad_norm_(policy.parameters(), max_grad_norm)
    policy.optimizer.step()          # the reference passes AdamW + weight_decay (train.py:125-142)
On the GPU that is ~60 small PyTorch launches per minibatch (per-tensor norms,
the foreach clip, capturable AdamW's per-tensor weight decay and bias
corrections).  `FlatAdamW` keeps the trainable parameters, exp_avg and
exp_avg_sq in three flat fp32 buffers (the parameters become views of the
first, each starting on a 16-byte boundary), copies the gradients into a
fourth (one foreach launch) and runs the clip and
the AdamW update in `bb_adamw_clip`: a single-workgroup norm/scalars launch and
one elementwise pass.  The math is torch.optim.AdamW's (amsgrad off) with
clip_grad_norm_'s factor min(1, max_norm / (||g|| + 1e-6)).

The learning rate lives in a device tensor (param_groups[0]["lr"]) so a captured
HIP graph replays every schedule value; `state[p]` exposes per-parameter views
of the moment buffers and the shared step counter, so snapshots and restores
work as with torch optimisers.  Raises if the native library is missing -- there
is no PyTorch fallback on the GPU.
"""
from __future__ import annotations

from typing import Iterable, List

import torch


def _ptr(t: torch.Tensor):
    return t.data_ptr()


class FlatAdamW:
    clips_grad = True  # the caller must not run clip_grad_norm_ itself

    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float, weight_decay: float, max_grad_norm: float,
                 betas=(0.9, 0.999), eps: float = 1e-8):
        from ballbot_gym import _native as N

        self._lib = N.lib()
        self._check = N.check
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("FlatAdamW: no trainable parameters")
        dev = self.params[0].device
        if dev.type != "cuda" or any(p.device != dev or p.dtype != torch.float32 for p in self.params):
            raise ValueError("FlatAdamW: fp32 parameters on one GPU expected")
        # every tensor starts on a 16-byte boundary (float4 loads in bb_ppo_mlp_step);
        # the gaps hold zeros in the parameter and gradient buffers
        self.offsets = []
        n = 0
        for p in self.params:
            self.offsets.append(n)
            n += (p.numel() + 3) // 4 * 4
        self.n = n
        self.flat = torch.zeros(n, device=dev)
        self.grad = torch.zeros(n, device=dev)
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.step_t = torch.zeros(1, device=dev)
        self.coef = torch.zeros(4, device=dev)
        self.lr = torch.tensor(float(lr), device=dev)
        self.beta1, self.beta2 = float(betas[0]), float(betas[1])
        self.eps, self.weight_decay, self.max_grad_norm = float(eps), float(weight_decay), float(max_grad_norm)
        self.state = {}
        self._gviews = []
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                k = p.numel()
                self.flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                self.state[p] = {"exp_avg": self.exp_avg[off:off + k].view_as(p),
                                 "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p), "step": self.step_t}
                self._gviews.append(self.grad[off:off + k].view_as(p))
        self.param_groups = [{"lr": self.lr, "params": self.params, "weight_decay": self.weight_decay,
                              "betas": (self.beta1, self.beta2), "eps": self.eps}]

    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params:
            if p.grad is None:
                continue
            if set_to_none:
                p.grad = None
            else:
                p.grad.zero_()

    def step(self) -> None:
        have = [(v, p.grad) for v, p in zip(self._gviews, self.params) if p.grad is not None]
        if have:
            torch._foreach_copy_([v for v, _ in have], [g for _, g in have])
        for v, p in zip(self._gviews, self.params):
            if p.grad is None:
                v.zero_()
        g = self.grad
        stream = torch.cuda.current_stream(self.flat.device).cuda_stream
        self._check(self._lib.bb_adamw_clip(_ptr(self.flat), _ptr(g), _ptr(self.exp_avg), _ptr(self.exp_avg_sq),
                                            int(self.n), _ptr(self.lr), _ptr(self.step_t), _ptr(self.coef),
                                            self.beta1, self.beta2, self.eps, self.weight_decay,
                                            self.max_grad_norm, stream), "bb_adamw_clip")
