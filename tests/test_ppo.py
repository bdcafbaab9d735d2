"""Trainer host logic on CPU: GAE restatement known answers,
schedule, policy structure, the BatchedPPO loop on a CPU stand-in env, log
columns vs the reference's progress.csv, and config -> PPO arguments."""
import json
import math
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import sb3_ref

GOLDEN = Path(__file__).parent / "golden"


def _torch_gae(rewards, values, starts, last_v, last_d, gamma, lam):
    a, r = sb3_ref.compute_gae(rewards.numpy(), values.numpy(), starts.numpy(), last_v.numpy(), last_d.numpy(),
                               gamma, lam)
    return torch.from_numpy(a), torch.from_numpy(r)


def test_gae_known_answers():
    rng = np.random.default_rng(0)
    T, N = 6, 3
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    starts = np.zeros((T, N), np.float32)
    dones = np.zeros(N, np.float32)
    g = 0.9
    # lambda = 1, no episode ends: A_t = sum_k g^(k-t) r_k + g^(T-t) V_T - V_t
    a, ret = sb3_ref.compute_gae(r, v, starts, lv, dones, g, 1.0)
    for t in range(T):
        mc = sum(g ** (k - t) * r[k].astype(np.float64) for k in range(t, T)) + g ** (T - t) * lv
        np.testing.assert_allclose(a[t], mc - v[t], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ret[t], mc, rtol=1e-5, atol=1e-5)
    # lambda = 0: one-step TD errors
    a0, _ = sb3_ref.compute_gae(r, v, starts, lv, dones, g, 0.0)
    nxt = np.concatenate([v[1:], lv[None]], 0)
    np.testing.assert_allclose(a0, r + g * nxt - v, rtol=1e-6, atol=1e-6)
    # an episode start at t=3 cuts the bootstrap of t=2; a last done cuts V_T
    starts[3, 1] = 1
    dones[2] = 1
    a1, _ = sb3_ref.compute_gae(r, v, starts, lv, dones, g, 0.0)
    assert a1[2, 1] == pytest.approx(r[2, 1] - v[2, 1], abs=1e-6)
    assert a1[T - 1, 2] == pytest.approx(r[T - 1, 2] - v[T - 1, 2], abs=1e-6)


def test_lr_schedule_reference_semantics():
    from ballbot_rl.training.schedules import lr_schedule

    assert lr_schedule(1.0) == 1e-4 and lr_schedule(0.71) == 1e-4
    assert lr_schedule(0.6) == 5e-5
    assert lr_schedule(0.7) == 1e-5  # strict comparisons in schedules.py:15-19
    assert lr_schedule(0.5) == 1e-5 and lr_schedule(0.0) == 1e-5


def test_policy_structure_and_distribution():
    from ballbot_rl.policies import ActorCriticPolicy, Extractor, obs_spaces

    sp = obs_spaces()
    assert list(sp) == ["actions", "angular_vel", "motor_state", "orientation", "vel"]
    cams = obs_spaces(cameras=True)
    assert list(cams) == ["actions", "angular_vel", "motor_state", "orientation", "relative_image_timestamp",
                          "rgbd_0", "rgbd_1", "vel"]
    assert Extractor(cams).features_dim == 15 + 1 + 20 + 20  # the paper's 56-d input
    torch.manual_seed(0)
    p = ActorCriticPolicy(sp)
    # 15 -> 128^4 per trunk, heads 3 and 1, log_std 3
    trunk = 15 * 128 + 128 + 3 * (128 * 128 + 128)
    assert sum(x.numel() for x in p.parameters()) == 2 * trunk + (128 * 3 + 3) + (128 + 1) + 3
    # orthogonal init with SB3 gains, zero biases
    w = p.policy_net[0].weight.detach()
    assert torch.allclose(w.T @ w, 2.0 * torch.eye(15), atol=1e-4)  # 128x15: orthonormal columns, gain^2 = 2
    assert float(p.action_net.weight.norm()) == pytest.approx(0.01 * math.sqrt(3), rel=1e-4)
    assert float(p.value_net.bias.abs().max()) == 0.0
    obs = torch.randn(32, 15)
    mean, _ = p._heads(obs)
    a = torch.randn(32, 3)
    ref = torch.distributions.Normal(mean, torch.exp(p.log_std)).log_prob(a).sum(-1)
    _, lp, ent = p.evaluate_actions(obs, a)
    assert torch.allclose(lp, ref, atol=1e-5)
    assert torch.allclose(ent, torch.distributions.Normal(mean, torch.exp(p.log_std)).entropy().sum(-1), atol=1e-6)
    d = {k: obs[:, 3 * i:3 * i + 3] for i, k in enumerate(sp)}
    assert torch.equal(p.features_extractor(d), p.features_extractor(obs))


def _ppo(env, **kw):
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    args = dict(n_steps=8, batch_size=32, n_epochs=2, ent_coef=0.001, clip_range=0.2, vf_coef=2.0, target_kl=None,
                learning_rate=3e-4, normalize_advantage=False, seed=1, gae_fn=_torch_gae,
                logger=CSVLogger(kw.pop("log_dir", None), stdout=False))
    args.update(kw)
    return BatchedPPO(env, **args)


def test_ppo_loop_on_cpu_stand_in(tmp_path):
    from fake_env import FakeEnv
    from ballbot_rl.training.logger import read_progress

    env = FakeEnv(16, ep_len=5)
    m = _ppo(env, log_dir=str(tmp_path))
    before = [p.detach().clone() for p in m.policy.parameters()]
    m.learn(total_timesteps=16 * 8 * 3)
    assert m.num_timesteps == 16 * 8 * 3
    assert m._n_updates == 3 * 2
    assert any(not torch.equal(a, b) for a, b in zip(before, m.policy.parameters()))
    # episodes of 5 steps (staggered start): completed lengths 5 except the first ones
    assert len(m.ep_info_buffer) > 0 and max(e["l"] for e in m.ep_info_buffer) == 5
    cols = read_progress(str(tmp_path / "progress.csv"))
    assert len(cols["time/total_timesteps"]) == 3
    assert cols["train/loss"][0] is None and cols["train/loss"][1] is not None  # train/* logged one dump later
    ref = set(json.loads((GOLDEN / "progress_columns.json").read_text())["columns"])
    eval_cols = {"eval/mean_ep_length", "eval/mean_reward"}
    assert set(cols) == ref - eval_cols  # eval/* come from the evaluation callback
    # the rollout stored unclipped actions; the env saw clipped ones
    assert float(m.buf.actions.abs().max()) <= 10


def test_ppo_kl_early_stop():
    from fake_env import FakeEnv

    env = FakeEnv(16)
    m = _ppo(env, target_kl=1e-12, learning_rate=1e-2, n_epochs=4)
    m.learn(total_timesteps=16 * 8 * 2)
    # first minibatch of the first epoch has KL 0 (same policy), later ones exceed 1.5 * target
    assert m._n_updates < 2 * 4


def test_ppo_kwargs_from_reference_config():
    from ballbot_rl.training.schedules import lr_schedule
    from ballbot_rl.training.train import ppo_kwargs

    cfg = {"algo": {"batch_sz": 256, "clip_range": 0.015, "ent_coef": 0.001, "learning_rate": -1, "n_epochs": 5,
                    "n_steps": 2048, "name": "ppo", "normalize_advantage": False, "target_kl": 0.3, "vf_coef": 2.0,
                    "weight_decay": 0.01}, "hidden_sz": 128}
    k = ppo_kwargs(cfg)
    assert k["learning_rate"] is lr_schedule
    assert (k["n_steps"], k["batch_size"], k["n_epochs"], k["clip_range"], k["target_kl"]) == (2048, 256, 5, 0.015, 0.3)
    assert k["net_arch"] == {"pi": [128] * 4, "vf": [128] * 4}


def test_training_config_loader(tmp_path):
    from ballbot_gym.core.config import get_component_config, load_training_config

    (tmp_path / "env").mkdir()
    (tmp_path / "train").mkdir()
    (tmp_path / "env" / "e.yaml").write_text("terrain: {type: perlin, config: {scale: 20.0}}\n"
                                             "reward: directional\nenv: {max_ep_steps: 100}\n")
    (tmp_path / "train" / "t.yaml").write_text("env_config: env/e.yaml\nalgo: {name: ppo}\nenv: {max_ep_steps: 50}\n")
    cfg = load_training_config(str(tmp_path / "train" / "t.yaml"))
    assert cfg["env"]["max_ep_steps"] == 50 and "env_config" not in cfg
    assert get_component_config(cfg, "terrain") == {"type": "perlin", "config": {"scale": 20.0}}
    assert get_component_config(cfg, "reward") == {"type": "directional", "config": {}}
    (tmp_path / "train" / "bad.yaml").write_text("algo: {name: ppo}\n")
    with pytest.raises(ValueError, match="env_config"):
        load_training_config(str(tmp_path / "train" / "bad.yaml"))
    with pytest.raises(ValueError, match="must have 'type'"):
        get_component_config({"reward": {"config": {}}}, "reward")


def test_encoder_roundtrip_and_frozen_extractor(tmp_path):
    """TinyAutoencoder (reference encoders/models.py) shapes, safetensors save/load with
    the p_sum check, and the frozen copies inside the Extractor."""
    from ballbot_rl.encoders import TinyAutoencoder, load_frozen_encoder, save_encoder
    from ballbot_rl.encoders.pretrain import train_autoencoder
    from ballbot_rl.policies import ActorCriticPolicy, obs_spaces

    torch.manual_seed(0)
    imgs = torch.rand(96, 1, 64, 64)
    ae = TinyAutoencoder(64, 64)
    assert ae(imgs[:4]).shape == (4, 1, 64, 64)
    path = str(tmp_path / "enc.safetensors")
    hist = train_autoencoder(ae, imgs, epochs=2, batch_size=32, save_path=path, log=lambda *_: None)
    assert np.isfinite(hist["best_val_loss"])
    enc = load_frozen_encoder(path)
    assert not any(p.requires_grad for p in enc.parameters())
    pol = ActorCriticPolicy(obs_spaces(cameras=True), frozen_encoder=enc)
    e0, e1 = pol.features_extractor.extractors["rgbd_0"], pol.features_extractor.extractors["rgbd_1"]
    assert e0 is not e1 and torch.equal(e0[0].weight, enc[0].weight)  # untouched by the orthogonal init
    assert pol.features_extractor.features_dim == 56
    import json
    meta = json.loads(open(path + ".json").read())
    meta["p_sum"] += 1.0
    open(path + ".json", "w").write(json.dumps(meta))
    with pytest.raises(ValueError, match="corrupted"):
        load_frozen_encoder(path)


def test_eval_callback_sb3_timing_targets_and_npz(tmp_path):
    """EvalCallback (callbacks.py:607-617 of the reference; SB3 semantics): an evaluation at
    every eval_freq-th vec-env step with the rollout's parameters, before its update; env i
    of the eval VecEnv counts (n_eval_episodes + i) // n_envs episodes, in finishing order;
    evaluations.npz as SB3 writes it (allow_pickle=False loads it); a progress.csv row with
    eval/* and time/total_timesteps."""
    from fake_env import FakeEnv
    from ballbot_rl.evaluation import evaluate_policy
    from ballbot_rl.training.callbacks import EvalCallback
    from ballbot_rl.training.logger import read_progress

    # targets over 10 envs and 8 episodes: [0, 0, 1, ..., 1] (SB3 evaluate_policy)
    ev = FakeEnv(10, seed=3, ep_len=4)
    policy = _ppo(FakeEnv(10), n_steps=4, batch_size=8).policy
    r = evaluate_policy(policy, ev, n_eval_episodes=8)
    assert len(r["episode_rewards"]) == 8 and len(r["episode_lengths"]) == 8
    assert all(l >= 1 for l in r["episode_lengths"])
    # staggered episodes: env i (i >= 2) ends its first episode after 4 - i % 4 steps; finishing order
    exp_len = sorted(((4 - i % 4) or 4, i) for i in range(2, 10))
    assert r["episode_lengths"] == [l for l, _ in exp_len]
    m = _ppo(FakeEnv(16, ep_len=5), n_steps=8, batch_size=32, log_dir=str(tmp_path))
    cb = EvalCallback(FakeEnv(16, seed=9, ep_len=6), n_eval_episodes=8, eval_freq=12, n_total_envs=16,
                      log_path=tmp_path / "results", best_model_save_path=tmp_path)
    calls = []
    m.learn(total_timesteps=16 * 8 * 5, rollout_callback=lambda mm, a, b: (calls.append((a, b)), cb(mm, a, b)))
    assert calls == [(1, 8), (9, 16), (17, 24), (25, 32), (33, 40)]
    d = np.load(tmp_path / "results" / "evaluations.npz", allow_pickle=False)
    assert d["timesteps"].tolist() == [12 * 16, 24 * 16, 36 * 16]  # vec-steps 12, 24, 36 x 16 envs
    assert d["results"].shape == (3, 8) and d["ep_lengths"].shape == (3, 8)
    cols = read_progress(str(tmp_path / "progress.csv"))
    evals = [v for v in cols["eval/mean_reward"] if v is not None]
    np.testing.assert_allclose(evals, d["results"].mean(1), rtol=1e-9)
    assert (tmp_path / "best_model.safetensors").exists()


def test_eval_callback_every_multiple_in_a_rollout(tmp_path):
    """eval_freq below n_steps: SB3's EvalCallback fires at every multiple of eval_freq inside
    one rollout (its _on_step runs per vec-env step), so a rollout of vec-steps [1, 8] with
    eval_freq 3 holds evaluations at 3 and 6, then 9, 12, 15 in the next, one npz row each."""
    from fake_env import FakeEnv
    from ballbot_rl.training.callbacks import EvalCallback

    cb = EvalCallback(FakeEnv(4, seed=2, ep_len=3), n_eval_episodes=4, eval_freq=3, n_total_envs=4,
                      log_path=tmp_path / "results")
    assert cb.due(1, 8) == [3, 6] and cb.due(9, 16) == [9, 12, 15] and cb.due(1, 2) == []
    m = _ppo(FakeEnv(4, ep_len=5), n_steps=8, batch_size=16, log_dir=str(tmp_path))
    m.learn(total_timesteps=4 * 8 * 2, rollout_callback=cb)
    d = np.load(tmp_path / "results" / "evaluations.npz", allow_pickle=False)
    assert d["timesteps"].tolist() == [12, 24, 36, 48, 60]
