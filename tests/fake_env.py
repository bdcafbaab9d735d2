"""A tiny CPU stand-in for BallbotVecEnv (test helper for the trainer's host logic).

Same interface: num_envs, device, reset() -> (obs[N,15], info), step(a[N,3]) ->
(obs, reward, terminated, truncated, info); episodes end after a fixed,
per-env staggered number of steps; reward favours a = clip(obs[:3]).
"""
import torch


class FakeEnv:
    def __init__(self, n, device="cpu", seed=0, ep_len=7):
        self.num_envs = n
        self.device = torch.device(device)
        self.g = torch.Generator().manual_seed(seed)
        self.ep_len = ep_len
        self.t = torch.arange(n) % ep_len
        self.obs = torch.zeros(n, 15)

    def reset(self):
        self.obs = torch.randn(self.num_envs, 15, generator=self.g)
        return self.obs, {}

    def step(self, a):
        target = self.obs[:, :3].clamp(-1, 1)
        r = (1.0 - ((a - target) ** 2).sum(1)).float()
        self.t += 1
        done = self.t >= self.ep_len
        self.t[done] = 0
        self.obs = torch.randn(self.num_envs, 15, generator=self.g)
        return self.obs, r, done, torch.zeros_like(done), {}

    def close(self):
        pass
