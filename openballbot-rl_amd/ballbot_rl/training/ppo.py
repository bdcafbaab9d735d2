"""Batched PPO on the GPU env.

Restates stable-baselines3 2.6.0 PPO as the reference configures it
(ballbot_rl/training/train.py:38-142, 284; configs/train/ppo_directional.yaml):

collect_rollouts (SB3 OnPolicyAlgorithm.collect_rollouts)
  n_steps env.steps of every env; actions are sampled from the Gaussian policy,
  CLIPPED to the action space [-1, 1] for env.step and stored UNCLIPPED;
  episode_starts[t] = done of the previous step; the reference env never
  truncates (ballbot_env.py:1030), so no time-limit bootstrap.
compute_returns_and_advantage -> bb_gae (HIP kernel, csrc/bb_rollout.hip).
train (SB3 PPO.train)
  n_epochs passes over random minibatches of batch_size; ratio = exp(logp -
  old_logp); clipped surrogate; value loss = MSE(returns, values) (no value
  clipping); entropy loss = -mean(entropy); loss = pg + ent_coef*ent +
  vf_coef*vf; approx_kl = mean(exp(r) - 1 - r) with r the log ratio, and the
  update STOPS (before the step) once approx_kl > 1.5 * target_kl; gradients
  clipped to max_grad_norm (0.5) by global norm; AdamW(weight_decay) with the
  learning rate from the schedule at progress_remaining = 1 - t/T.
Logs: SB3's keys and order (training/logger.py), rollout stats over the last 100
episodes (Monitor + ep_info_buffer).

Everything stays on the GPU: rollout buffers [T][N] in HBM, one host sync per
rollout for episode statistics and one per minibatch for the KL early stop
(SB3's semantics need it).  Multi-GPU: each rank
steps its own env shard; at the update boundary the rollout buffers are
gathered to rank 0 over RCCL (gather_rollouts), rank 0 runs the update and
broadcasts the new parameters (update_mode="gather", north_star's design and
the default).  update_mode="allreduce" instead updates data-parallel: every rank takes its minibatches (batch_size / world rows each)
from its own shard, the advantages are normalised over the global minibatch, the
gradients are averaged with an RCCL all-reduce before the clip and AdamW step,
and the KL early stop uses the ranks' mean approx_kl, so no rank waits for rank
0.  The all-reduces are nodes of the captured per-minibatch / per-epoch update
graphs (with the fused minibatch split around them, bb_ppo_mlp_args.phase); the
eager minibatch loop is the fallback (use_graphs=False, a short last minibatch).
"""
from __future__ import annotations

import ctypes as C
import os
import time
from collections import deque
from typing import Any, Callable, Dict, Optional, Union

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from ballbot_rl.policies.mlp_policy import ActorCriticPolicy, obs_spaces
from ballbot_rl.training.logger import CSVLogger

Schedule = Union[float, Callable[[float], float]]


def _ptr(t: torch.Tensor):
    return C.c_void_p(t.data_ptr())


_DEBUG_GRAPHS = os.environ.get("BB_DEBUG_GRAPHS", "0") != "0"


def _dbg(msg: str) -> None:
    """BB_DEBUG_GRAPHS=1: synchronize and log each graph phase (locates an asynchronous fault)."""
    if _DEBUG_GRAPHS:
        torch.cuda.synchronize()
        print(f"[graphs] ok: {msg}", flush=True)


def gae_hip(rewards, values, episode_starts, last_values, last_dones, gamma: float, gae_lambda: float):
    """GAE on device tensors [T][N] through the C-ABI (bb_gae); raises off-GPU."""
    from ballbot_gym import _native as N

    if not rewards.is_cuda:
        raise RuntimeError("bb_gae runs on the GPU; rollout tensors must live on a ROCm device")
    T, n = rewards.shape
    ts = [rewards, values, episode_starts, last_values, last_dones]
    want = [(torch.float32, (T, n)), (torch.float32, (T, n)), (torch.uint8, (T, n)), (torch.float32, (n,)),
            (torch.uint8, (n,))]
    for t, (dt, sh) in zip(ts, want):
        if t.dtype != dt or tuple(t.shape) != sh or not t.is_contiguous():
            raise ValueError(f"bb_gae: expected contiguous {dt} {sh}, got {t.dtype} {tuple(t.shape)}")
    adv = torch.empty_like(rewards)
    ret = torch.empty_like(rewards)
    stream = C.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    N.check(N.lib().bb_gae(*[_ptr(t) for t in ts], int(T), int(n), float(gamma), float(gae_lambda), _ptr(adv),
                           _ptr(ret), stream), "bb_gae")
    return adv, ret


class _PPOLossHIP(torch.autograd.Function):
    """bb_ppo_loss: the SB3 minibatch loss and its gradients in one HIP launch.

    forward -> (loss, pg, vf, ent, approx_kl, clip_fraction); backward scales the
    gradients the kernel already wrote (d loss / d mean, values, log_std)."""

    @staticmethod
    def forward(ctx, mean, values, log_std, actions, old_logp, adv, ret, clip_t, normalize, ent_coef, vf_coef):
        from ballbot_gym import _native as N

        B = mean.shape[0]
        terms = torch.empty(9, device=mean.device, dtype=torch.float32)
        gmean = torch.empty_like(mean)
        gval = torch.empty_like(values)
        ts = [t.contiguous() for t in (mean, values, log_std, actions, old_logp, adv, ret, clip_t)]
        stream = C.c_void_p(torch.cuda.current_stream(mean.device).cuda_stream)
        N.check(N.lib().bb_ppo_loss(*[_ptr(t) for t in ts], int(B), int(normalize), float(ent_coef),
                                    float(vf_coef), _ptr(terms), _ptr(gmean), _ptr(gval), stream), "bb_ppo_loss")
        ctx.save_for_backward(gmean, gval, terms)
        aux = terms[1:6].clone()
        ctx.mark_non_differentiable(aux)
        return terms[0].clone(), aux

    @staticmethod
    def backward(ctx, g_loss, _g_terms):
        gmean, gval, terms = ctx.saved_tensors
        return (g_loss * gmean, g_loss * gval, g_loss * terms[6:9], None, None, None, None, None, None, None, None)


def explained_variance(y_pred: torch.Tensor, y_true: torch.Tensor) -> float:
    """SB3 common.utils.explained_variance: 1 - Var[y - y_pred] / Var[y] (nan if Var[y] == 0)."""
    var_y = torch.var(y_true, unbiased=False)
    if float(var_y) == 0:
        return float("nan")
    return float(1.0 - torch.var(y_true - y_pred, unbiased=False) / var_y)


class RolloutBuffer:
    """[T][N] device buffers of one rollout (SB3 RolloutBuffer, device-resident)."""

    def __init__(self, T: int, n: int, obs_dim: int, act_dim: int, device, image_shape=None):
        f32 = dict(dtype=torch.float32, device=device)
        self.T, self.n = T, n
        self.obs = torch.zeros(T, n, obs_dim, **f32)
        # depth cameras (F2): [T][N][2][H][W] images + relative_image_timestamp
        self.depth = torch.zeros(T, n, *image_shape, **f32) if image_shape else None
        self.rel_ts = torch.zeros(T, n, **f32) if image_shape else None
        self.actions = torch.zeros(T, n, act_dim, **f32)
        self.rewards = torch.zeros(T, n, **f32)
        self.values = torch.zeros(T, n, **f32)
        self.log_probs = torch.zeros(T, n, **f32)
        self.starts = torch.zeros(T, n, dtype=torch.uint8, device=device)
        self.advantages = None
        self.returns = None

    def flat(self) -> Dict[str, torch.Tensor]:
        """Flattened [T*N] views (the sample order does not matter: minibatches are random)."""
        T, n = self.T, self.n
        d = {"obs": self.obs.reshape(T * n, -1), "actions": self.actions.reshape(T * n, -1),
             "values": self.values.reshape(-1), "log_probs": self.log_probs.reshape(-1),
             "advantages": self.advantages.reshape(-1), "returns": self.returns.reshape(-1)}
        if self.depth is not None:
            d["depth"] = self.depth.reshape(T * n, *self.depth.shape[2:])
            d["rel_ts"] = self.rel_ts.reshape(-1)
        return d


def policy_obs(obs15: torch.Tensor, depth: Optional[torch.Tensor] = None,
               rel_ts: Optional[torch.Tensor] = None):
    """The policy's observation: the packed proprio tensor, or with cameras the
    reference's key dict (ballbot_env.py:812-826) the Extractor concatenates."""
    if depth is None:
        return obs15
    d = {k: obs15[:, 3 * i:3 * i + 3] for i, k in enumerate(("actions", "angular_vel", "motor_state",
                                                             "orientation", "vel"))}
    d["rgbd_0"] = depth[:, 0:1]
    d["rgbd_1"] = depth[:, 1:2]
    d["relative_image_timestamp"] = rel_ts.reshape(-1, 1)
    return d


def fused_mlp_slots(ppo: "BatchedPPO", update: bool = True, B: Optional[int] = None):
    """Flat-buffer offsets of the 21 tensors bb_ppo_mlp_step reads, or None when
    the policy/optimiser is not the reference's MLP on FlatAdamW (pi = vf =
    [128]*4 LeakyReLU(0.01) over the 15-d proprio obs, or the 56-d features of
    the camera policy with fused frozen encoders; 3-d action head);
    update=True also needs a minibatch bb_ppo_mlp_step takes: B rows (default
    ppo.batch_size; the data-parallel update passes its local batch_size / world),
    a multiple of 256 in [256, 16384] -- else the autograd graph step runs.
    BB_PPO_FUSED=0 disables the fused update and rollout step (A/B runs)."""
    import os

    from ballbot_rl.training.optim import FlatAdamW

    if os.environ.get("BB_PPO_FUSED", "1") == "0" or ppo.device.type != "cuda":
        return None
    opt, pol = ppo.optimizer, ppo.policy
    if not isinstance(opt, FlatAdamW):
        return None
    if update:  # the LOCAL minibatch bb_ppo_mlp_step runs: batch_size / world rows when data-parallel
        B = int(ppo.batch_size if B is None else B)
        if B < 256 or B % 256 or B > 16384:
            return None

    ext = pol.features_extractor
    fd = ext.features_dim
    if ppo.cameras:  # the camera features must come from fused frozen encoders (no trainable extractor)
        keys, frozen = getattr(ext, "keys", None), getattr(ext, "_frozen_keys", None)
        if keys is None or frozen is None:  # a custom extractor: the autograd path
            return None
        rgbd = {k for k in keys if "rgbd_" in k}
        order = ["actions", "angular_vel", "motor_state", "orientation", "relative_image_timestamp", "rgbd_0", "rgbd_1",
                 "vel"]  # the feature layout _UpdateGraphs assembles for the fused minibatch
        if fd != 56 or keys != order or frozen != rgbd or any(p.requires_grad for p in ext.parameters()):
            return None
    elif fd != 15:
        return None

    def trunk(seq):
        mods = list(seq)
        if len(mods) != 8:
            return None
        lins, acts = mods[0::2], mods[1::2]
        shapes = [(128, fd), (128, 128), (128, 128), (128, 128)]
        if any(not isinstance(m, nn.Linear) or m.bias is None or tuple(m.weight.shape) != sh
               for m, sh in zip(lins, shapes)):
            return None
        if any(not isinstance(a, nn.LeakyReLU) or a.negative_slope != 0.01 for a in acts):
            return None
        return [m.weight for m in lins] + [m.bias for m in lins]

    pi, vf = trunk(pol.policy_net), trunk(pol.value_net_trunk)
    if pi is None or vf is None:
        return None
    if tuple(pol.action_net.weight.shape) != (3, 128) or tuple(pol.value_net.weight.shape) != (1, 128):
        return None
    tensors = pi + vf + [pol.action_net.weight, pol.action_net.bias, pol.value_net.weight, pol.value_net.bias,
                         pol.log_std]
    where = {id(q): off for q, off in zip(opt.params, opt.offsets)}
    if len(opt.params) != len(tensors) or any(id(t) not in where for t in tensors):
        return None
    return [where[id(t)] for t in tensors]


class _UpdateGraphs:
    """PPO.train as ONE captured graph per minibatch, replayed with no host sync.

    The graph reads minibatch `k` of a static permutation (device counter),
    evaluates the SB3 loss terms into a log row, back-propagates, and runs
    clip_grad_norm_ + AdamW (capturable).  SB3's KL early stop (break BEFORE the
    step once approx_kl > 1.5 * target_kl, ending the update) is applied
    optimistically: all epochs replay back to back, one host sync reads the log
    rows, and if some row r tripped the stop the policy and AdamW state are
    restored from the snapshot taken at the start and rows 0..r-1 are replayed
    again with the same permutations -- the exact steps SB3 takes.  The stop is
    rare (approx_kl ~1e-3 against 0.45 in the reference's runs), so the common
    update costs no sync at all.  Requires n % batch_size == 0 (SB3's short last
    minibatch goes through the eager path)."""

    LOG_COLS = 6  # loss, pg, vf, ent, kl, clip_fraction

    def __init__(self, ppo: "BatchedPPO", n: int, B: Optional[int] = None):
        dev = ppo.device
        B = ppo.batch_size if B is None else int(B)
        # data-parallel update (update_mode="allreduce"): each minibatch's graph also holds the
        # ranks' all-reduces -- the global advantage statistics before the loss, the gradient
        # between backward and the clip + AdamW step (RCCL collectives captured in the graph)
        self.dp = ppo._dp
        self.B = B
        self.n, self.nb = n, n // B
        self.data = {"obs": torch.zeros(n, 15, device=dev), "actions": torch.zeros(n, 3, device=dev),
                     "log_probs": torch.zeros(n, device=dev), "advantages": torch.zeros(n, device=dev),
                     "returns": torch.zeros(n, device=dev)}
        if ppo.cameras:
            self.data["depth"] = torch.zeros(n, 2, ppo.env.cam_h, ppo.env.cam_w, device=dev)
            self.data["rel_ts"] = torch.zeros(n, device=dev)
        self.perm = torch.zeros(self.nb, B, dtype=torch.int64, device=dev)
        self.perms = torch.zeros(ppo.n_epochs, self.nb, B, dtype=torch.int64, device=dev)
        self.k = torch.zeros(1, dtype=torch.int64, device=dev)        # minibatch within the epoch
        self.row = torch.zeros(1, dtype=torch.int64, device=dev)      # log row within the update
        self.clip = torch.zeros((), device=dev)
        self.adv_stats = torch.zeros(2, device=dev)  # dp: the global minibatch's mean, 1 / (std + 1e-8)
        self.log = torch.zeros(ppo.n_epochs * self.nb, self.LOG_COLS, device=dev)
        self.params = params = [p for p in ppo.policy.parameters() if p.requires_grad]
        # BatchNorm running statistics and num_batches_tracked of the (frozen) encoders: a
        # train-mode minibatch moves them, so the warm-up/capture below and the KL-stop
        # replay must restore them with the parameters
        self.buffers = [b for b in ppo.policy.buffers()]
        opt = ppo.optimizer
        p_snap = [p.detach().clone() for p in params]
        st_snap = {id(p): {k: v.clone() for k, v in opt.state[p].items()} for p in params if p in opt.state}
        b_snap = [b.detach().clone() for b in self.buffers]

        slots = fused_mlp_slots(ppo, B=B)
        self.fused = slots is not None
        if self.fused:
            mb_step = self._fused_step(ppo, slots)
        else:
            mb_step = self._autograd_step(ppo, params, opt)
        self.perm.copy_(torch.arange(self.nb * B, device=dev).view(self.nb, B) % max(n, 1))
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up (also creates the AdamW state the graph updates)
                self.k.zero_(); self.row.zero_()
                mb_step()
        torch.cuda.current_stream(dev).wait_stream(side)
        for p in params:  # backward allocates the grads inside the graph pool (static addresses)
            p.grad = None
        self.k.zero_(); self.row.zero_()
        # thread-local capture: with RCCL collectives in the graph, the process group's watchdog
        # thread polls the events of the warm-up's (eager) collectives while this thread captures;
        # under the default global mode that poll invalidates the capture (hipErrorStreamCapture-
        # Invalidated, seen on one GPU with an RCCL group in round 6, tests/test_gpu_rccl.py)
        mode = "thread_local"
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode=mode):
            mb_step()
        # the fused proprio minibatch advances its own device counters, so a whole epoch
        # (nb minibatches) is one graph as well: one host launch per epoch instead of nb
        self.graph_epoch = None
        if self.fused and "depth" not in self.data and self.nb > 1:
            self.graph_epoch = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_epoch, capture_error_mode=mode):
                for _ in range(self.nb):
                    mb_step()
        torch.cuda.synchronize(dev)
        self._restore(opt, [p_snap, {i: st_snap.get(id(p)) for i, p in enumerate(params)}, b_snap])
        _dbg(f"update graphs built (fused={self.fused}, epoch graph={self.graph_epoch is not None})")

    def prime(self, ppo: "BatchedPPO") -> None:
        """Replay each captured graph once on the static zero data and restore the parameters,
        AdamW state and BatchNorm statistics: a graph's first replay uploads it (~50 ms for the
        update's graphs), which would otherwise land in the first update of learn()."""
        opt = ppo.optimizer
        snap = self._snapshot(opt)
        for g in (self.graph, self.graph_epoch):
            if g is not None:
                self.k.zero_(); self.row.zero_()
                g.replay()
        torch.cuda.synchronize(ppo.device)
        self._restore(opt, snap)
        self.k.zero_(); self.row.zero_(); self.log.zero_()

    def _fused_step(self, ppo: "BatchedPPO", slots):
        """bb_ppo_mlp_step: the whole minibatch (forward, loss, backward, clip,
        AdamW) in five HIP launches; it advances k and row itself."""
        from ballbot_gym import _native as N

        opt, lib = ppo.optimizer, N.lib()
        nbytes = C.c_int64()
        N.check(lib.bb_ppo_mlp_workspace_bytes(int(ppo.batch_size), C.byref(nbytes)), "bb_ppo_mlp_workspace_bytes")
        self.ws = torch.empty(int(nbytes.value) // 4, device=ppo.device)
        a = N.PPOMlpArgs()
        a.params, a.grad, a.exp_avg, a.exp_avg_sq = (t.data_ptr() for t in (opt.flat, opt.grad, opt.exp_avg,
                                                                            opt.exp_avg_sq))
        a.n_params = int(opt.n)
        for i, o in enumerate(slots):
            a.offsets[i] = int(o)
        d = self.data
        cams = "depth" in d
        fd = ppo.policy.features_extractor.features_dim
        if cams:  # the minibatch's features (frozen encoders in train mode) land here, in minibatch order
            self.feats = torch.zeros(self.B, fd, device=ppo.device)
        a.obs = self.feats.data_ptr() if cams else d["obs"].data_ptr()
        a.obs_dim, a.obs_direct = int(fd), int(cams)
        a.actions, a.old_logp = d["actions"].data_ptr(), d["log_probs"].data_ptr()
        a.advantages, a.returns = d["advantages"].data_ptr(), d["returns"].data_ptr()
        a.perm, a.mb_counter, a.row_counter, a.log = (t.data_ptr() for t in (self.perm, self.k, self.row, self.log))
        a.clip, a.lr, a.step, a.coef = (t.data_ptr() for t in (self.clip, opt.lr, opt.step_t, opt.coef))
        a.B = int(self.B)
        a.normalize_advantage = int(ppo.normalize_advantage)
        dp_norm = self.dp and ppo.normalize_advantage
        a.adv_stats = self.adv_stats.data_ptr() if dp_norm else None
        a.ent_coef, a.vf_coef = float(ppo.ent_coef), float(ppo.vf_coef)
        a.beta1, a.beta2, a.eps = opt.beta1, opt.beta2, opt.eps
        a.weight_decay, a.max_grad_norm = opt.weight_decay, opt.max_grad_norm
        a.workspace, a.workspace_bytes = self.ws.data_ptr(), int(nbytes.value)
        self._args = a
        dev = ppo.device

        ext = ppo.policy.features_extractor

        def mb_step():
            if cams:  # the Extractor's sorted-key concatenation, the images read through idx by the kernel
                from ballbot_rl.encoders.models import fused_encoder_forward

                idx = self.perm.index_select(0, self.k).view(-1)
                o15 = d["obs"][idx]
                f = self.feats
                f[:, 0:12].copy_(o15[:, 0:12])              # actions, angular_vel, motor_state, orientation
                f[:, 12].copy_(d["rel_ts"][idx])            # relative_image_timestamp
                for c, key in enumerate(("rgbd_0", "rgbd_1")):
                    f[:, 13 + 20 * c:33 + 20 * c].copy_(
                        fused_encoder_forward(ext.extractors[key], d["depth"][:, c:c + 1], index=idx))
                f[:, 53:56].copy_(o15[:, 12:15])            # vel
            stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            if not self.dp:
                a.phase = 0
                N.check(lib.bb_ppo_mlp_step(C.byref(a), stream), "bb_ppo_mlp_step")
                return
            if dp_norm:
                self._global_adv_stats(ppo)
            a.phase = 1  # forward, loss, backward: the flat gradient, the log row, the counters
            N.check(lib.bb_ppo_mlp_step(C.byref(a), stream), "bb_ppo_mlp_step")
            ppo._allreduce(opt.grad)  # the ranks' mean gradient
            opt.grad.div_(ppo.world)
            a.phase = 2  # clip + AdamW over the mean gradient
            N.check(lib.bb_ppo_mlp_step(C.byref(a), stream), "bb_ppo_mlp_step")

        return mb_step

    def _global_adv_stats(self, ppo: "BatchedPPO") -> None:
        """The global minibatch's advantage mean and 1 / (std + 1e-8) into adv_stats (SB3's
        normalisation over the union of the ranks' local minibatches: one all-reduce of count,
        sum and sum of squares, fp64), read by the fused tile kernel (bb_ppo_mlp_args.adv_stats)."""
        idx = self.perm.index_select(0, self.k).view(-1)
        a64 = self.data["advantages"][idx].double()
        t = torch.stack([torch.full((), float(a64.numel()), dtype=torch.float64, device=a64.device), a64.sum(),
                         (a64 * a64).sum()])
        ppo._allreduce(t)
        mean = t[1] / t[0]
        var = (t[2] - t[0] * mean * mean) / torch.clamp(t[0] - 1.0, min=1.0)
        std = torch.sqrt(torch.clamp(var, min=0.0))
        self.adv_stats.copy_(torch.stack([mean, 1.0 / (std + 1e-8)]).float())

    def _autograd_step(self, ppo: "BatchedPPO", params, opt):
        def mb_step():
            d = self.data
            idx = self.perm.index_select(0, self.k).view(-1)
            adv, norm = d["advantages"][idx], None
            if self.dp and ppo.normalize_advantage:  # the global minibatch's normalisation
                adv, norm = ppo._global_normalized(adv), False
            loss, pg, vf, ent, kl, cf = ppo._loss(ppo._mb_obs(d, idx), d["actions"][idx], d["log_probs"][idx],
                                                  adv, d["returns"][idx], self.clip, normalize=norm)
            self.log.index_copy_(0, self.row, torch.stack([loss.detach(), pg, vf, ent, kl, cf]).view(1, -1))
            for p in params:
                if p.grad is not None:
                    p.grad.zero_()
            loss.backward()
            if self.dp:  # the ranks' mean gradient before the clip and the step
                ppo._allreduce_grads(params)
            if not getattr(opt, "clips_grad", False):
                nn.utils.clip_grad_norm_(params, ppo.max_grad_norm)
            opt.step()
            with torch.no_grad():
                self.k.add_(1)
                self.row.add_(1)

        return mb_step

    def _snapshot(self, opt):
        return [[p.detach().clone() for p in self.params],
                {i: {k: v.clone() for k, v in opt.state[p].items()} for i, p in enumerate(self.params)},
                [b.detach().clone() for b in self.buffers]]

    def _restore(self, opt, snap) -> None:
        with torch.no_grad():
            for p, s_ in zip(self.params, snap[0]):
                p.copy_(s_)
            for i, p in enumerate(self.params):
                prev = snap[1].get(i)
                for k, v in opt.state[p].items():
                    if prev is not None and k in prev:
                        v.copy_(prev[k])
                    else:
                        v.zero_()
            for b, s_ in zip(self.buffers, snap[2]):
                b.copy_(s_)

    @torch.no_grad()
    def _stats_forward(self, ppo: "BatchedPPO", row: int) -> None:
        """SB3 evaluates the minibatch that trips the KL stop (train mode) before it
        breaks: its BatchNorm statistics move once more, with no optimiser step."""
        if not self.buffers:
            return
        e, k = divmod(row, self.nb)
        idx = self.perms[e][k]
        d = self.data
        if self.fused and "depth" in d:
            from ballbot_rl.encoders.models import fused_encoder_forward

            ext = ppo.policy.features_extractor
            for c, key in enumerate(("rgbd_0", "rgbd_1")):
                fused_encoder_forward(ext.extractors[key], d["depth"][:, c:c + 1], index=idx)
        else:
            ppo.policy.features_extractor(ppo._mb_obs(d, idx))

    def _replay(self, rows: int) -> None:
        self.row.zero_()
        done = 0
        for e in range(self.perms.shape[0]):
            if done >= rows:
                break
            self.perm.copy_(self.perms[e])
            self.k.zero_()
            if self.graph_epoch is not None and rows - done >= self.nb:
                self.graph_epoch.replay()
                done += self.nb
                continue
            for _ in range(min(self.nb, rows - done)):
                self.graph.replay()
                done += 1

    def run(self, ppo: "BatchedPPO", d: Dict[str, torch.Tensor], clip: float):
        """All epochs of one update; -> the log rows SB3 would have recorded, [rows, 6] on the host."""
        for k, v in self.data.items():
            v.copy_(d[k])
        self.clip.fill_(clip)
        for e in range(ppo.n_epochs):
            self.perms[e].copy_(torch.randperm(self.n, generator=ppo.shuffle_gen, device=ppo.device).view(self.nb, -1))
        total = ppo.n_epochs * self.nb
        snap = self._snapshot(ppo.optimizer) if ppo.target_kl is not None else None
        _dbg("update: before replay")
        self._replay(total)
        _dbg("update: replayed")
        if self.dp and ppo._collective:  # the global minibatches' terms: the ranks' mean (the KL stop reads it)
            ppo._allreduce(self.log)
            self.log.div_(ppo.world)
        log = self.log.cpu().numpy()
        if ppo.target_kl is not None:
            trip = np.nonzero(log[:, 4] > 1.5 * ppo.target_kl)[0]
            if len(trip):
                r = int(trip[0])
                ppo.kl_stops += 1  # an update that replays: restore + r minibatches again
                self._restore(ppo.optimizer, snap)
                self._replay(r)            # the steps before the tripping minibatch
                self._stats_forward(ppo, r)  # ... and its own forward (BatchNorm statistics)
                keep = log[:r + 1].copy()  # ... whose own terms SB3 still logs
                return keep
        return log


class _RolloutGraph:
    """One proprio rollout -- n_steps x (bb_ppo_mlp_act, env.step_flags, bb_rollout_track)
    -- captured as ONE HIP graph and replayed once per rollout (SB3 collect_rollouts).

    A captured graph keeps the raw device pointers of everything its kernels read
    and write.  Every such buffer is therefore owned here (the Gaussian noise, the
    clipped actions, the finished-episode rows) or is a fixed buffer of the env,
    the rollout buffer or the optimiser that lives as long as the graph.  The eager
    loop allocates noise / clipped / ep_r / ep_l afresh per rollout: a capture of
    that loop bakes in the first rollout's addresses, which the caching allocator
    hands to other tensors -- or unmaps (empty_cache, an allocation retry under
    memory pressure) -- once the rollout's tensors are freed, so a later replay
    reads stale memory or faults with an illegal address.  That is how the
    round-2 per-step capture could fault only when other tests ran beside it.
    The env's step (routing, both step kernels on two streams) is captured as in
    BallbotVecEnv.capture_step; the handle's counters and lists are written by
    the graph's kernels in stream order, as in eager stepping."""

    def __init__(self, ppo: "BatchedPPO", slots):
        from ballbot_gym import _native as N

        env, b, dev = ppo.env, ppo.buf, ppo.device
        T, n = ppo.n_steps, ppo.n_envs
        self.env, self.key = env, (id(env), T, n)
        self.noise = torch.zeros(T, n, 3, device=dev)
        self.clipped = torch.zeros(n, 3, device=dev)
        self.ep_r = torch.zeros(T, n, dtype=torch.float64, device=dev)
        self.ep_l = torch.zeros(T, n, dtype=torch.int64, device=dev)
        self.flat = ppo.optimizer.flat
        self.offs = (C.c_int32 * 21)(*slots)
        lib = N.lib()
        obs = env.obs  # step_flags returns the env's own observation buffer: read in place
        flat, nflat = C.c_void_p(self.flat.data_ptr()), int(self.flat.numel())
        torch.cuda.synchronize(dev)
        _dbg(f"rollout graph: capture T={T} n={n} obs={obs.data_ptr():#x} flat={self.flat.data_ptr():#x}")
        env.note_graph_capture()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            b.starts[0].copy_(ppo._last_starts)
            for t in range(T):
                N.check(lib.bb_ppo_mlp_act(flat, self.offs, nflat, _ptr(obs), 15, _ptr(self.noise[t]), n,
                                           _ptr(b.obs[t]), _ptr(b.actions[t]), _ptr(self.clipped),
                                           _ptr(b.values[t]), _ptr(b.log_probs[t]), stream), "bb_ppo_mlp_act")
                o, reward, flags = env.step_flags(self.clipped)
                if o.data_ptr() != obs.data_ptr() or not reward.is_contiguous():
                    raise RuntimeError("rollout graph: env.step_flags must return its fixed buffers")
                nxt = _ptr(b.starts[t + 1]) if t + 1 < T else None
                N.check(lib.bb_rollout_track(_ptr(reward), _ptr(flags), 1, n, _ptr(b.rewards[t]),
                                             _ptr(ppo._ep_ret), _ptr(ppo._ep_len), _ptr(self.ep_r[t]),
                                             _ptr(self.ep_l[t]), _ptr(ppo._last_starts), nxt, stream),
                        "bb_rollout_track")
        torch.cuda.synchronize(dev)
        _dbg("rollout graph: captured")

    def run(self, ppo: "BatchedPPO"):
        if ppo._last_obs.data_ptr() != self.env.obs.data_ptr():
            self.env.obs.copy_(ppo._last_obs)
        self.noise.normal_(generator=ppo.gen)  # == torch.randn(T, n, 3, generator=gen): the eager draws
        _dbg("rollout graph: before replay")
        self.graph.replay()
        _dbg("rollout graph: replayed")
        ppo._last_obs = self.env.obs
        return self.ep_r, self.ep_l


class BatchedPPO:
    """PPO with SB3's arguments and defaults, over a batched GPU env.

    env: BallbotVecEnv-like object with num_envs, device, reset() -> (obs, info)
    and step(actions) -> (obs, reward, terminated, truncated, info), obs a
    packed [N, 15] tensor.  Rollout length per env is n_steps, so one rollout
    holds num_envs * n_steps samples."""

    def __init__(self, env, learning_rate: Schedule = 3e-4, n_steps: int = 2048, batch_size: int = 64,
                 n_epochs: int = 10, gamma: float = 0.99, gae_lambda: float = 0.95, clip_range: Schedule = 0.2,
                 normalize_advantage: bool = True, ent_coef: float = 0.0, vf_coef: float = 0.5,
                 max_grad_norm: float = 0.5, target_kl: Optional[float] = None, weight_decay: float = 0.01,
                 net_arch: Optional[Dict[str, Any]] = None, activation_fn=nn.LeakyReLU, seed: int = 0,
                 logger: Optional[CSVLogger] = None, stats_window_size: int = 100,
                 gae_fn: Callable = gae_hip, policy: Optional[ActorCriticPolicy] = None,
                 use_graphs: Optional[bool] = None, frozen_encoder: Optional[nn.Module] = None,
                 update_mode: Optional[str] = None):
        self.env = env
        self.device = torch.device(env.device)
        self.n_envs = int(env.num_envs)
        self.n_steps, self.batch_size, self.n_epochs = int(n_steps), int(batch_size), int(n_epochs)
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        self.lr_schedule = learning_rate if callable(learning_rate) else (lambda _p, v=float(learning_rate): v)
        self.clip_schedule = clip_range if callable(clip_range) else (lambda _p, v=float(clip_range): v)
        self.normalize_advantage = bool(normalize_advantage)
        self.ent_coef, self.vf_coef, self.max_grad_norm = float(ent_coef), float(vf_coef), float(max_grad_norm)
        self.target_kl = None if target_kl is None else float(target_kl)
        self.gae_fn = gae_fn
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        # RCCL process group (backend "nccl"): the collectives run even at world size 1, so a one-GPU
        # run executes the same captured all-reduce nodes as the multi-GPU one
        self._rccl = bool(dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl")
        if update_mode is None:  # north_star's design: rollouts gathered to rank 0 at the update boundary
            update_mode = "gather"
        if update_mode not in ("gather", "allreduce"):
            raise ValueError(f"update_mode must be 'gather' or 'allreduce' (got {update_mode!r})")
        if update_mode == "allreduce" and self.world > 1 and int(batch_size) % self.world:
            raise ValueError(f"update_mode='allreduce': batch_size {batch_size} must divide by the {self.world} ranks")
        if update_mode == "allreduce" and self.world > 1:
            # every rank must run the same number of minibatches (one all-reduce each): equal
            # shards, or the collectives stop matching (gloo errors, RCCL hangs)
            dev = torch.device("cpu") if dist.get_backend() == "gloo" else self.device
            t = torch.tensor([self.n_envs, -self.n_envs], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if int(t[0]) != self.n_envs or int(-t[1]) != self.n_envs:
                raise ValueError(f"update_mode='allreduce' needs the same number of envs on every rank (this rank "
                                 f"has {self.n_envs}, the ranks range over [{int(-t[1])}, {int(t[0])}]): make "
                                 "num_envs divisible by the world size")
        self.update_mode = update_mode
        # the data-parallel update; _force_dp runs it at world size 1 too (tests: its collectives
        # are then the identity, so its graph is checked against the eager form on one GPU)
        self._force_dp = False
        self.kl_stops = 0  # updates the KL early stop ended (diagnostic: each replays part of the update)
        self._dp_adv_hook = None  # tests: called with each data-parallel minibatch's normalised advantages
        torch.manual_seed(int(seed))
        self.cameras = bool(getattr(env, "cameras", False))
        img = (2, env.cam_h, env.cam_w) if self.cameras else None
        spaces = obs_spaces(cameras=True, height=env.cam_h, width=env.cam_w) if self.cameras else obs_spaces()
        self.policy = (policy or ActorCriticPolicy(spaces, 3, net_arch, activation_fn,
                                                   frozen_encoder=frozen_encoder)).to(self.device)
        self._sync_params()
        # full-size minibatches replay one HIP graph (forward+backward, clip+AdamW).
        # On the GPU clip_grad_norm_ + AdamW are bb_adamw_clip over flat buffers
        # (FlatAdamW, learning rate in a device tensor); on the CPU torch's AdamW
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else bool(use_graphs)
        lr0 = self.lr_schedule(1.0)
        if self.device.type == "cuda":
            from ballbot_rl.training.optim import FlatAdamW

            self.optimizer = FlatAdamW(self.policy.parameters(), lr=lr0, weight_decay=float(weight_decay),
                                       max_grad_norm=self.max_grad_norm)
        else:
            self.optimizer = torch.optim.AdamW(self.policy.parameters(), lr=lr0, weight_decay=float(weight_decay))
        self._graphs = None
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed) * 1000003 + self.rank)
        self.shuffle_gen = torch.Generator(device=self.device)
        self.shuffle_gen.manual_seed(int(seed) + 7)
        self.logger = logger or CSVLogger(None, stdout=False)
        self.buf = RolloutBuffer(self.n_steps, self.n_envs, 15, 3, self.device, img)
        self.num_timesteps = 0
        self._n_updates = 0
        self.ep_info_buffer: deque = deque(maxlen=int(stats_window_size))
        self._last_obs = None
        self._last_starts = torch.ones(self.n_envs, dtype=torch.uint8, device=self.device)
        self._ep_ret = torch.zeros(self.n_envs, dtype=torch.float64, device=self.device)
        self._ep_len = torch.zeros(self.n_envs, dtype=torch.int64, device=self.device)
        self.progress_remaining = 1.0
        self._act_slots = None  # fused rollout policy step: slots, False (not eligible) or None (not checked)
        self._rgraph: Optional[_RolloutGraph] = None

    # ------------------------------------------------------------ distributed
    def _sync_params(self) -> None:
        if self.world == 1:
            return
        vec = nn.utils.parameters_to_vector(self.policy.parameters()).detach().contiguous()
        dist.broadcast(vec, src=0)
        with torch.no_grad():  # in place: FlatAdamW's parameters are views of its flat buffer
            off = 0
            for p in self.policy.parameters():
                k = p.numel()
                p.copy_(vec[off:off + k].view_as(p))
                off += k

    # ---------------------------------------------------------------- rollout
    def _collect_fused(self, slots) -> tuple:
        if self.cameras:
            return self._collect_fused_cameras(slots)
        return self._collect_fused_proprio(slots)

    def _collect_fused_cameras(self, slots) -> tuple:
        """The camera policy's rollout: features from the Extractor (fused frozen
        encoders, eval mode), then bb_ppo_mlp_act on the 56-d features and
        bb_rollout_track; the rollout buffer keeps obs, images and timestamps."""
        from ballbot_gym import _native as N

        env, b, dev = self.env, self.buf, self.device
        lib = N.lib()
        T, n = self.n_steps, self.n_envs
        offs = (C.c_int32 * 21)(*slots)
        flat = C.c_void_p(self.optimizer.flat.data_ptr())
        nflat = int(self.optimizer.flat.numel())
        ext = self.policy.features_extractor
        self.policy.eval()
        if self._last_obs is None:
            self._last_obs, _ = env.reset()
        noise = torch.randn(T, n, 3, generator=self.gen, device=dev)
        clipped = torch.empty(n, 3, device=dev)
        ep_r = torch.empty(T, n, dtype=torch.float64, device=dev)
        ep_l = torch.empty(T, n, dtype=torch.int64, device=dev)
        b.starts[0].copy_(self._last_starts)
        stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        # The cameras re-render an env every 6 steps (and at its reset): exactly the envs whose
        # relative_image_timestamp is 0.  In eval mode the encoder is a fixed function of the
        # image, so the other envs keep last step's camera features (bit-identical); the cache
        # is rebuilt at every rollout start (the update moved the BatchNorm statistics).
        from ballbot_rl.encoders.models import fused_encoder_forward

        cache = os.environ.get("BB_ENC_CACHE", "1") != "0"
        feats = torch.empty(n, 56, device=dev)
        encs = (ext.extractors["rgbd_0"], ext.extractors["rgbd_1"])
        for t in range(T):
            b.obs[t].copy_(self._last_obs)
            b.depth[t].copy_(env.depth)
            b.rel_ts[t].copy_(env.rel_ts)
            feats[:, 0:12].copy_(b.obs[t][:, 0:12])
            feats[:, 12].copy_(b.rel_ts[t])
            feats[:, 53:56].copy_(b.obs[t][:, 12:15])
            idx = None if (t == 0 or not cache) else torch.nonzero(b.rel_ts[t] == 0).view(-1)
            if idx is None:
                for c, enc in enumerate(encs):
                    feats[:, 13 + 20 * c:33 + 20 * c].copy_(fused_encoder_forward(enc, b.depth[t][:, c:c + 1]))
            elif idx.numel():
                for c, enc in enumerate(encs):
                    f = fused_encoder_forward(enc, b.depth[t][:, c:c + 1], index=idx)
                    feats[:, 13 + 20 * c:33 + 20 * c].index_copy_(0, idx, f)
            N.check(lib.bb_ppo_mlp_act(flat, offs, nflat, _ptr(feats), int(feats.shape[1]), _ptr(noise[t]), n, None,
                                       _ptr(b.actions[t]), _ptr(clipped), _ptr(b.values[t]), _ptr(b.log_probs[t]),
                                       stream), "bb_ppo_mlp_act")
            obs, reward, flags = env.step_flags(clipped)
            nxt = _ptr(b.starts[t + 1]) if t + 1 < T else None
            N.check(lib.bb_rollout_track(_ptr(reward.contiguous()), _ptr(flags), 1, n, _ptr(b.rewards[t]),
                                         _ptr(self._ep_ret), _ptr(self._ep_len), _ptr(ep_r[t]), _ptr(ep_l[t]),
                                         _ptr(self._last_starts), nxt, stream), "bb_rollout_track")
            self._last_obs = obs
        return ep_r, ep_l

    def _collect_rollout_kernel(self, slots) -> tuple:
        """The whole proprio rollout as ONE launch (bb_rollout): every env runs its
        n_steps of (policy, sample, clip, env step, bookkeeping) back to back on
        its team.  Same buffers and noise draws as the per-step fused rollout; the
        policy sums in another fp32 order than bb_ppo_mlp_act's MFMA tiles
        (tests/test_gpu_rollout.py)."""
        from ballbot_gym import _native as N

        env, b, dev = self.env, self.buf, self.device
        T, n = self.n_steps, self.n_envs
        if self._last_obs is None:
            self._last_obs, _ = env.reset()
        obs_io = env.obs
        if self._last_obs.data_ptr() != obs_io.data_ptr():
            obs_io.copy_(self._last_obs)
        noise = torch.randn(T, n, 3, generator=self.gen, device=dev)
        # "no episode ended" in every row before the launch: a relief-pair rollout that ends on
        # its budget leaves rows unwritten, and those must not read as finished episodes
        ep_r = torch.full((T, n), float("nan"), dtype=torch.float64, device=dev)
        ep_l = torch.zeros(T, n, dtype=torch.int64, device=dev)
        # bb_rollout reads the trunk weights input-major (W^T): a transposed copy per rollout
        flat = self.optimizer.flat
        if getattr(self, "_pol_t", None) is None or self._pol_t.numel() != flat.numel():
            self._pol_t = torch.empty_like(flat)
        pt = self._pol_t
        pt.copy_(flat)
        for w0 in (0, 8):  # MLP_PI_W0, MLP_VF_W0 (bb_mlp.h)
            for l in range(4):
                o, k = int(slots[w0 + l]), (15 if l == 0 else 128)
                pt[o:o + 128 * k].view(k, 128).copy_(flat[o:o + 128 * k].view(128, k).t())
        a = N.RolloutArgs()
        a.params, a.n_params, a.noise, a.n_steps = pt.data_ptr(), int(pt.numel()), noise.data_ptr(), T
        for i, o in enumerate(slots):
            a.offsets[i] = int(o)
        a.obs, a.last_starts = obs_io.data_ptr(), self._last_starts.data_ptr()
        a.ep_ret, a.ep_len = self._ep_ret.data_ptr(), self._ep_len.data_ptr()
        a.buf_obs, a.buf_actions, a.buf_values = b.obs.data_ptr(), b.actions.data_ptr(), b.values.data_ptr()
        a.buf_log_prob, a.buf_rewards, a.buf_starts = b.log_probs.data_ptr(), b.rewards.data_ptr(), b.starts.data_ptr()
        a.ep_r_out, a.ep_l_out = ep_r.data_ptr(), ep_l.data_ptr()
        env.run_rollout(a)
        if getattr(env, "relief", False):  # the relief pair's budget fault, before GAE and the update
            env.check()                    # read the buffer (the rollout's host sync comes next anyway)
        self._last_obs = obs_io
        return ep_r, ep_l

    def _collect_fused_proprio(self, slots) -> tuple:
        """collect_rollouts with the policy step as bb_ppo_mlp_act and the
        episode bookkeeping as bb_rollout_track: three launches per env step
        (policy, bb_step, bookkeeping) instead of ~40.  Same semantics as the
        torch loop below (tests/test_gpu_ppo.py: test_fused_rollout_matches_torch)."""
        from ballbot_gym import _native as N

        env, b, dev = self.env, self.buf, self.device
        lib = N.lib()
        T, n = self.n_steps, self.n_envs
        if self._last_obs is None:
            self._last_obs, _ = env.reset()
        # the whole rollout as one bb_rollout launch (on relief banks the relief pair with the
        # policy in it): 4096 perlin envs on per-env generators, 64-step rollouts, 67 ms per
        # rollout against 81 ms for the per-step graph below (tools/archive/r5_pair_rollout.sh).
        # BB_FUSED_ROLLOUT=0 forces the per-step form.
        fr = os.environ.get("BB_FUSED_ROLLOUT", "auto")
        if hasattr(env, "run_rollout") and getattr(env, "_host_reward", None) is None and fr != "0":
            return self._collect_rollout_kernel(slots)
        if (self.use_graphs and hasattr(env, "step_flags") and getattr(env, "_host_reward", None) is None
                and hasattr(env, "obs") and os.environ.get("BB_ROLLOUT_GRAPH", "1") != "0"):
            if self._rgraph is None or self._rgraph.key != (id(env), T, n):
                self._rgraph = _RolloutGraph(self, slots)
            return self._rgraph.run(self)
        offs = (C.c_int32 * 21)(*slots)
        flat = C.c_void_p(self.optimizer.flat.data_ptr())
        nflat = int(self.optimizer.flat.numel())
        noise = torch.randn(T, n, 3, generator=self.gen, device=dev)
        clipped = torch.empty(n, 3, device=dev)
        ep_r = torch.empty(T, n, dtype=torch.float64, device=dev)
        ep_l = torch.empty(T, n, dtype=torch.int64, device=dev)
        b.starts[0].copy_(self._last_starts)
        fast = hasattr(env, "step_flags")
        stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for t in range(T):
            obs_in = self._last_obs.contiguous()
            N.check(lib.bb_ppo_mlp_act(flat, offs, nflat, _ptr(obs_in), 15, _ptr(noise[t]), n, _ptr(b.obs[t]),
                                       _ptr(b.actions[t]),
                                       _ptr(clipped), _ptr(b.values[t]), _ptr(b.log_probs[t]), stream),
                    "bb_ppo_mlp_act")
            if fast:
                obs, reward, flags = env.step_flags(clipped)
                mask = 1  # BB_DONE_TERMINATED (the reference never truncates; a divergence reset ends nothing)
            else:
                obs, reward, term, trunc, _info = env.step(clipped)
                flags, mask = (term | trunc).to(torch.uint8).contiguous(), 1
            reward = reward.contiguous()
            nxt = _ptr(b.starts[t + 1]) if t + 1 < T else None
            N.check(lib.bb_rollout_track(_ptr(reward), _ptr(flags), mask, n, _ptr(b.rewards[t]), _ptr(self._ep_ret),
                                         _ptr(self._ep_len), _ptr(ep_r[t]), _ptr(ep_l[t]), _ptr(self._last_starts),
                                         nxt, stream), "bb_rollout_track")
            self._last_obs = obs
        return ep_r, ep_l

    @torch.no_grad()
    def collect_rollouts(self) -> None:
        env, b = self.env, self.buf
        if self._act_slots is None and self.device.type == "cuda":
            self._act_slots = fused_mlp_slots(self, update=False) or False
        if self._act_slots and (not self.cameras or hasattr(env, "step_flags")):
            ep_r, ep_l = self._collect_fused(self._act_slots)
            self._finish_rollout(ep_r, ep_l)
            return
        self.policy.eval()  # SB3 set_training_mode(False): BatchNorm uses running stats
        if self._last_obs is None:
            self._last_obs, _ = env.reset()
        ep_r, ep_l = [], []
        # the rollout's Gaussian draws in one launch (SB3 samples per step; same distribution)
        noise = torch.randn(self.n_steps, self.n_envs, 3, generator=self.gen, device=self.device)
        for t in range(self.n_steps):
            b.obs[t].copy_(self._last_obs)        # env.obs is reused by the next step
            b.starts[t].copy_(self._last_starts)
            if self.cameras:
                b.depth[t].copy_(env.depth)
                b.rel_ts[t].copy_(env.rel_ts)
                pobs = policy_obs(b.obs[t], b.depth[t], b.rel_ts[t])
            else:
                pobs = b.obs[t]
            actions, values, logp = self.policy(pobs, noise=noise[t])
            b.actions[t].copy_(actions)
            b.values[t].copy_(values)
            b.log_probs[t].copy_(logp)
            obs, reward, term, trunc, info = env.step(actions.clamp(-1.0, 1.0))
            flags = info.get("done_flags") if isinstance(info, dict) else None
            done = (term | trunc) if flags is None else ((flags & 1) != 0) | trunc
            b.rewards[t].copy_(reward)
            self._ep_ret += reward.double()
            self._ep_len += 1
            ep_r.append(torch.where(done, self._ep_ret, torch.full_like(self._ep_ret, float("nan"))))
            ep_l.append(torch.where(done, self._ep_len, torch.zeros_like(self._ep_len)))
            self._ep_ret.masked_fill_(done, 0.0)
            self._ep_len.masked_fill_(done, 0)
            self._last_obs = obs
            self._last_starts = done.to(torch.uint8)
        self._finish_rollout(torch.stack(ep_r), torch.stack(ep_l))

    def _finish_rollout(self, ep_r: torch.Tensor, ep_l: torch.Tensor) -> None:
        """GAE and the finished episodes ([T][N] returns, NaN where none ended; lengths)."""
        env, b = self.env, self.buf
        self.num_timesteps += self.n_envs * self.n_steps * self.world
        last_v = self.policy.predict_values(
            policy_obs(self._last_obs, env.depth, env.rel_ts) if self.cameras else self._last_obs)
        b.advantages, b.returns = self.gae_fn(b.rewards, b.values, b.starts, last_v.contiguous(),
                                              self._last_starts.contiguous(), self.gamma, self.gae_lambda)
        # finished episodes in time order (one host sync per rollout)
        r = ep_r.cpu().numpy()
        ln = ep_l.cpu().numpy()
        mask = ~np.isnan(r)
        finished = list(zip(r[mask].tolist(), ln[mask].tolist()))
        if self.world > 1:
            parts = [None] * self.world
            dist.all_gather_object(parts, finished)
            finished = [x for p in parts for x in p]
        for rr, ll in finished:
            self.ep_info_buffer.append({"r": rr, "l": ll})

    # ----------------------------------------------------------------- update
    def _gathered(self) -> Optional[Dict[str, torch.Tensor]]:
        d = self.buf.flat()
        if self.world == 1:
            return d
        from ballbot_gym.distributed import gather_rollouts

        out = {}
        for k, v in d.items():  # [T*n, ...] per rank -> concatenated on rank 0
            g = gather_rollouts(v.unsqueeze(0))
            out[k] = None if g is None else g.reshape(-1, *v.shape[1:])
        return out if self.rank == 0 else None

    def _graphs_for(self, n: int, bsz: Optional[int] = None) -> Optional[_UpdateGraphs]:
        bsz = self.batch_size if bsz is None else int(bsz)
        if n < bsz or n % bsz:
            return None
        if self._graphs is None or self._graphs.n != n or self._graphs.B != bsz or self._graphs.dp != self._dp:
            self._graphs = _UpdateGraphs(self, n, bsz)
        return self._graphs

    def train(self) -> None:
        if self._dp:
            self._update(self.buf.flat(), dp=True)  # every rank, its own shard; parameters stay equal
            if self.world > 1:
                for bf in self.policy.buffers():  # BatchNorm statistics (camera encoder) from rank 0
                    dist.broadcast(bf, src=0)
            return
        data = self._gathered()
        if data is not None:
            self._update(data)
        self._sync_params()

    @property
    def _dp(self) -> bool:
        return self.update_mode == "allreduce" and (self._collective or self._force_dp)

    @property
    def _collective(self) -> bool:
        """The update's collectives execute: several ranks, or an RCCL group of any size."""
        return self.world > 1 or self._rccl

    def _allreduce(self, t: torch.Tensor) -> None:
        """Sum t over the ranks in place (RCCL on the GPU; captured when inside a graph); the
        identity on one rank without an RCCL group."""
        if self._collective:
            dist.all_reduce(t)

    def _allreduce_grads(self, params) -> None:
        """Average the parameters' gradients over the ranks: one all-reduce of the flattened set."""
        if not self._collective:
            return
        gs = [p_.grad for p_ in params if p_.grad is not None]
        fg = torch._utils._flatten_dense_tensors(gs)
        dist.all_reduce(fg)
        fg.div_(self.world)
        for g_, f_ in zip(gs, torch._utils._unflatten_dense_tensors(fg, gs)):
            g_.copy_(f_)

    def _allreduce_mean(self, ts) -> list:
        """The ranks' mean of several scalars, in ONE all-reduce."""
        t = torch.stack([x.detach().float().reshape(()) for x in ts])
        self._allreduce(t)
        return list(t / self.world)

    def _global_normalized(self, adv: torch.Tensor) -> torch.Tensor:
        """SB3's per-minibatch advantage normalisation, (adv - mean) / (std + 1e-8)
        with the unbiased std, over the GLOBAL minibatch: the union of the ranks'
        local minibatches (one all-reduce of count, sum and sum of squares)."""
        a64 = adv.detach().double()
        t = torch.stack([torch.full((), float(a64.numel()), dtype=torch.float64, device=adv.device), a64.sum(),
                         (a64 * a64).sum()])
        self._allreduce(t)
        n, s1, s2 = t[0], t[1], t[2]  # device scalars: no host sync (graph-capturable)
        mean = s1 / n
        var = (s2 - n * mean * mean) / torch.clamp(n - 1.0, min=1.0)
        std = torch.sqrt(torch.clamp(var, min=0.0))
        out = ((a64 - mean) / (std + 1e-8)).to(adv.dtype)
        if self._dp_adv_hook is not None:
            self._dp_adv_hook(adv, out)
        return out

    def _loss(self, obs, act, old_logp, adv, ret, clip, normalize: Optional[bool] = None):
        """One minibatch of SB3 PPO.train: -> (loss, pg, vf, ent, approx_kl, clip_fraction).

        On the GPU the loss and its gradients are one bb_ppo_loss launch; the
        torch expression below is the CPU stand-in path of the host tests.
        normalize: override of normalize_advantage (False: adv is normalised already)."""
        norm = self.normalize_advantage if normalize is None else bool(normalize)
        if self.device.type == "cuda":
            mean, values = self.policy._heads(obs)
            clip_t = clip if isinstance(clip, torch.Tensor) else torch.tensor(float(clip), device=self.device)
            loss, t = _PPOLossHIP.apply(mean, values, self.policy.log_std, act, old_logp, adv, ret, clip_t,
                                        norm, self.ent_coef, self.vf_coef)
            return loss, t[0], t[1], t[2], t[3], t[4]
        values, logp, entropy = self.policy.evaluate_actions(obs, act)
        if norm and adv.shape[0] > 1:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        log_ratio = logp - old_logp
        ratio = torch.exp(log_ratio)
        pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
        vf = nn.functional.mse_loss(ret, values)
        ent = -torch.mean(entropy)
        loss = pg + self.ent_coef * ent + self.vf_coef * vf
        with torch.no_grad():
            kl = torch.mean((ratio - 1) - log_ratio)
            cf = torch.mean((torch.abs(ratio - 1) > clip).float())
        return loss, pg.detach(), vf.detach(), ent.detach(), kl, cf

    def _mb_obs(self, d: Dict[str, torch.Tensor], idx: torch.Tensor):
        if "depth" in d:
            return policy_obs(d["obs"][idx], d["depth"][idx], d["rel_ts"][idx])
        return d["obs"][idx]

    def _update(self, d: Dict[str, torch.Tensor], dp: bool = False) -> None:
        """SB3 PPO.train over the rollout d.  dp: data-parallel over the ranks
        (update_mode="allreduce"): local minibatches of batch_size / world rows,
        gradients averaged over the ranks before the step, the KL stop on the
        ranks' mean approx_kl (eager minibatches: the all-reduce sits between
        backward and step)."""
        self.policy.train()
        lr = self.lr_schedule(self.progress_remaining)
        clip = self.clip_schedule(self.progress_remaining)
        n = d["obs"].shape[0]
        for g in self.optimizer.param_groups:
            if isinstance(g["lr"], torch.Tensor):
                g["lr"].fill_(lr)
            else:
                g["lr"] = lr
        bsz = self.batch_size // self.world if dp else self.batch_size
        # a data-parallel update captures its all-reduces in the graphs: RCCL ("nccl") collectives
        # can be captured, gloo's (CPU) cannot -- the eager loop then runs them
        dp_graph = not dp or self.world == 1 or dist.get_backend() == "nccl"
        graphs = self._graphs_for(n, bsz) if self.use_graphs and dp_graph else None
        loss = torch.zeros((), device=self.device)
        ent_l, pg_l, vf_l, clip_f, kls = [], [], [], [], []
        if graphs is not None:
            log = graphs.run(self, d, clip)
            nb = graphs.nb
            for e in range(self.n_epochs):
                rows = log[e * nb:(e + 1) * nb]
                if len(rows) == 0:
                    break
                self._n_updates += 1
                kls = rows[:, 4].tolist()
                for r in rows:
                    pg_l.append(torch.tensor(r[1])); vf_l.append(torch.tensor(r[2])); ent_l.append(torch.tensor(r[3]))
                    clip_f.append(torch.tensor(r[5]))
                loss = torch.tensor(rows[-1, 0])
        else:
            cont = True
            for _epoch in range(self.n_epochs):
                kls = []
                perm = torch.randperm(n, generator=self.shuffle_gen, device=self.device)
                for s in range(0, n, bsz):
                    idx = perm[s:s + bsz]
                    adv = d["advantages"][idx]
                    norm = None
                    if dp and self.normalize_advantage:  # SB3 normalises over the (global) minibatch
                        adv, norm = self._global_normalized(adv), False
                    loss, pg, vf, ent, kl, cf = self._loss(self._mb_obs(d, idx), d["actions"][idx],
                                                           d["log_probs"][idx], adv, d["returns"][idx], clip,
                                                           normalize=norm)
                    if dp:  # the global minibatch's terms: the mean over the ranks' local minibatches
                        pg, vf, ent, kl, cf = self._allreduce_mean((pg, vf, ent, kl, cf))
                    pg_l.append(pg); vf_l.append(vf); ent_l.append(ent); clip_f.append(cf)
                    approx_kl = float(kl)  # the early stop needs it before the step (host sync)
                    kls.append(approx_kl)
                    if self.target_kl is not None and approx_kl > 1.5 * self.target_kl:
                        cont = False
                        break
                    self.optimizer.zero_grad(set_to_none=False)
                    loss.backward()
                    if dp:  # average the gradient over the ranks: one all-reduce (RCCL on the GPU)
                        self._allreduce_grads(self.policy.parameters())
                    if not getattr(self.optimizer, "clips_grad", False):
                        nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
                    self.optimizer.step()
                self._n_updates += 1
                if not cont:
                    break
        L = self.logger
        mean = lambda xs: float(torch.stack(xs).mean()) if xs else float("nan")  # noqa: E731
        L.record("train/entropy_loss", mean(ent_l))
        L.record("train/policy_gradient_loss", mean(pg_l))
        L.record("train/value_loss", mean(vf_l))
        L.record("train/approx_kl", float(np.mean(kls)) if kls else float("nan"))  # last epoch, as SB3
        L.record("train/clip_fraction", mean(clip_f))
        L.record("train/loss", float(loss.detach()))
        L.record("train/explained_variance", explained_variance(d["values"], d["returns"]))
        L.record("train/std", float(torch.exp(self.policy.log_std.detach()).mean()))
        L.record("train/n_updates", self._n_updates)
        L.record("train/clip_range", clip)
        L.record("train/learning_rate", lr)

    def warm_up(self) -> "BatchedPPO":
        """Build, before learn(), what its first iteration would otherwise build inside the run:
        the update graphs of this trainer's update shape (_UpdateGraphs: two warm-up minibatches,
        the captures and one replay of each graph on static zero data, after which the
        parameters, AdamW state and BatchNorm statistics are restored; the first BLAS call of the
        bootstrap value; the first device randperm and reductions of the update, on a throwaway
        generator).  The training trajectory is unchanged
        (tests/test_gpu_ppo.py::test_warm_up_keeps_the_trajectory).  SB3 builds its model in the
        constructor (_setup_model); this is the same kind of setup, kept out of the constructor so
        that a trainer that never learns does not pay for it."""
        if self.device.type != "cuda" or not self.use_graphs:
            return self
        n_local = self.n_envs * self.n_steps
        was_training = self.policy.training
        self.policy.train()  # _update captures in train mode (BatchNorm of the camera encoders)
        g = None
        if self._dp:
            if self.world == 1 or dist.get_backend() == "nccl":
                g = self._graphs_for(n_local, self.batch_size // self.world)
        elif self.rank == 0:
            g = self._graphs_for(n_local * self.world)
        if g is not None:
            g.prime(self)
        # the rollout's bootstrap value is a torch forward: its first GEMM initialises the BLAS
        # library (~0.2 s), so run one here
        self.policy.eval()
        with torch.no_grad():
            o = torch.zeros(self.n_envs, 15, device=self.device)
            self.policy.predict_values(policy_obs(o, self.env.depth, self.env.rel_ts) if self.cameras else o)
            # the update's first calls of torch kernels outside the graphs: the minibatch shuffle
            # (a device randperm of the update's rows: a sort) and explained_variance's reductions,
            # on a throwaway generator so that shuffle_gen's stream is untouched
            n_upd = n_local if self._dp else n_local * self.world
            torch.randperm(n_upd, generator=torch.Generator(device=self.device).manual_seed(0), device=self.device)
            explained_variance(torch.zeros(n_upd, device=self.device),
                               torch.arange(n_upd, dtype=torch.float32, device=self.device))
            float(torch.exp(self.policy.log_std.detach()).mean())  # train/std's elementwise kernels
        self.policy.train(was_training)
        torch.cuda.synchronize(self.device)
        return self

    # ------------------------------------------------------------------ learn
    def learn(self, total_timesteps: int, callback: Optional[Callable[["BatchedPPO"], bool]] = None,
              log_interval: int = 1,
              rollout_callback: Optional[Callable[["BatchedPPO", int, int], None]] = None) -> "BatchedPPO":
        """SB3 OnPolicyAlgorithm.learn: rollout -> (logs) -> update until total_timesteps.
        rollout_callback(self, first_vec_step, last_vec_step): after each rollout and
        before its update, with the parameters the rollout ran with -- where SB3's
        per-step callbacks (EvalCallback's _on_step) see them; callback(self): after
        the update."""
        total = int(total_timesteps)
        t0 = time.perf_counter()
        start_steps = self.num_timesteps
        iteration = 0
        while self.num_timesteps < total:
            v0 = self.num_timesteps // max(self.n_envs * self.world, 1)
            self.collect_rollouts()
            if rollout_callback is not None:
                rollout_callback(self, v0 + 1, v0 + self.n_steps)
            iteration += 1
            self.progress_remaining = 1.0 - float(self.num_timesteps) / float(total)
            if log_interval and iteration % log_interval == 0 and self.rank == 0:
                el = max(time.perf_counter() - t0, 1e-9)
                L = self.logger
                L.record("time/iterations", iteration)
                if self.ep_info_buffer:
                    L.record("rollout/ep_rew_mean", float(np.mean([e["r"] for e in self.ep_info_buffer])))
                    L.record("rollout/ep_len_mean", float(np.mean([e["l"] for e in self.ep_info_buffer])))
                L.record("time/fps", int((self.num_timesteps - start_steps) / el))
                L.record("time/time_elapsed", int(el))
                L.record("time/total_timesteps", self.num_timesteps)
                L.dump(step=self.num_timesteps)
            self.train()
            if callback is not None and callback(self) is False:
                break
        return self

    # ------------------------------------------------------------- save/load
    def save(self, path: str) -> None:
        """Policy weights as safetensors (no pickle) + hyperparameters as JSON."""
        import json

        from safetensors.torch import save_file

        save_file({k: v.detach().contiguous().cpu() for k, v in self.policy.state_dict().items()}, path)
        meta = {"num_timesteps": self.num_timesteps, "n_updates": self._n_updates, "gamma": self.gamma,
                "gae_lambda": self.gae_lambda, "n_steps": self.n_steps, "batch_size": self.batch_size,
                "n_epochs": self.n_epochs}
        with open(str(path) + ".json", "w") as f:
            json.dump(meta, f)

    def load_policy(self, path: str) -> None:
        from safetensors.torch import load_file

        self.policy.load_state_dict(load_file(path, device=str(self.device)))
        self._sync_params()
