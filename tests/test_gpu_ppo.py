"""GPU: bb_gae bit-exact vs the SB3 restatement, and the batched PPO trainer on
the real env."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import sb3_ref  # noqa: E402


@pytest.mark.parametrize("T,N,p_done", [(64, 4096, 0.02), (1, 300, 0.5), (17, 1000, 0.0), (33, 77, 1.0)])
def test_gae_kernel_bit_exact(T, N, p_done):
    from ballbot_rl.training.ppo import gae_hip

    rng = np.random.default_rng(T * 1000 + N)
    r = rng.normal(0, 1, (T, N)).astype(np.float32)
    v = rng.normal(0, 3, (T, N)).astype(np.float32)
    st = (rng.random((T, N)) < p_done).astype(np.uint8)
    lv = rng.normal(0, 3, N).astype(np.float32)
    ld = (rng.random(N) < p_done).astype(np.uint8)
    dev = torch.device("cuda:0")
    a, ret = gae_hip(*(torch.from_numpy(x).to(dev) for x in (r, v, st, lv, ld)), 0.99, 0.95)
    ea, er = sb3_ref.compute_gae(r, v, st, lv, ld, 0.99, 0.95)
    assert np.array_equal(a.cpu().numpy(), ea), np.abs(a.cpu().numpy() - ea).max()
    assert np.array_equal(ret.cpu().numpy(), er)


def test_gae_rejects_bad_layout():
    from ballbot_rl.training.ppo import gae_hip

    dev = torch.device("cuda:0")
    z = torch.zeros(4, 8, device=dev)
    with pytest.raises(ValueError):
        gae_hip(z, z, torch.zeros(4, 8, device=dev), z[0], torch.zeros(8, dtype=torch.uint8, device=dev), .99, .95)


def test_batched_ppo_on_gpu_env(tmp_path):
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger, read_progress
    from ballbot_rl.training.ppo import BatchedPPO

    env = BallbotVecEnv(1024, device="cuda:0", max_ep_steps=10, seed=3)  # episodes end inside the run
    m = BatchedPPO(env, n_steps=16, batch_size=4096, n_epochs=2, ent_coef=0.001, clip_range=0.015, vf_coef=2.0,
                   target_kl=0.3, learning_rate=1e-4, normalize_advantage=False, seed=10,
                   logger=CSVLogger(str(tmp_path), stdout=False))
    m.learn(total_timesteps=1024 * 16 * 3)
    assert m.num_timesteps == 1024 * 16 * 3
    cols = read_progress(str(tmp_path / "progress.csv"))
    assert all(np.isfinite(x) for x in cols["train/loss"][1:])
    assert cols["rollout/ep_len_mean"][-1] > 0
    assert torch.isfinite(m.buf.advantages).all() and torch.isfinite(m.buf.returns).all()
    env.close()


def test_train_main_end_to_end(tmp_path):
    """train.main on the reference's flat-directional config (GPU-sized num_envs/n_steps)."""
    from ballbot_rl.training.train import main

    cfg = {"algo": {"batch_sz": 2048, "clip_range": 0.015, "ent_coef": 0.001, "learning_rate": -1, "n_epochs": 2,
                    "n_steps": 8, "name": "ppo", "normalize_advantage": False, "target_kl": 0.3, "vf_coef": 2.0,
                    "weight_decay": 0.01},
           "env": {"max_allowed_tilt": 20, "max_ep_steps": 100, "max_wheel_velocity": 10.0},
           "evaluation": {"freq": 8, "n_episodes": 4}, "hidden_sz": 64, "num_envs": 512, "seed": 10,
           "problem": {"reward": {"type": "directional", "config": {"target_direction": [0.0, 1.0]}},
                       "terrain": {"type": "flat", "config": {}}}, "total_timesteps": 512 * 8 * 2}
    m = main(cfg, 10, out=str(tmp_path / "run"))
    out = m.out_path
    for f in ("config.yaml", "info.txt", "progress.csv", "final_model.safetensors", "best_model.safetensors"):
        assert (out / f).exists(), f
    from ballbot_rl.training.logger import read_progress

    cols = read_progress(str(out / "progress.csv"))
    assert "eval/mean_reward" in cols


@pytest.mark.parametrize("target_kl", [None, 2e-4])
def test_graph_update_matches_eager(target_kl, monkeypatch):
    """The graph-replayed update (device-side KL stop) == the eager SB3 update on the same rollout
    (autograd minibatches on both sides; the fused minibatch has its own tests below)."""
    monkeypatch.setenv("BB_PPO_FUSED", "0")
    from fake_env import FakeEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    dev = torch.device("cuda:0")

    class GpuFake(FakeEnv):
        def __init__(self):
            super().__init__(256, ep_len=6)
            self.device = dev

        def reset(self):
            o, i = super().reset()
            return o.to(dev), i

        def step(self, a):
            o, r, d, t, i = super().step(a.cpu())
            return o.to(dev), r.to(dev), d.to(dev), t.to(dev), i

    models = []
    for graphs in (False, True):
        m = BatchedPPO(GpuFake(), n_steps=16, batch_size=512, n_epochs=3, learning_rate=1e-3, target_kl=target_kl,
                       normalize_advantage=True, seed=4, use_graphs=graphs, logger=CSVLogger(None, stdout=False))
        m.collect_rollouts()
        models.append(m)
    d0 = models[0].buf.flat()
    for m in models:  # same rollout data and shuffles for both
        m.shuffle_gen.manual_seed(99)
        m._update({k: v.clone() for k, v in d0.items()})
    assert models[1]._graphs is not None
    assert models[0]._n_updates == models[1]._n_updates
    if target_kl is not None:
        assert models[0]._n_updates < 3  # the stop fired
    for a, b in zip(models[0].policy.parameters(), models[1].policy.parameters()):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()
    la, lb = models[0].logger.values, models[1].logger.values
    for k in ("train/policy_gradient_loss", "train/value_loss", "train/approx_kl", "train/clip_fraction"):
        assert la[k] == pytest.approx(lb[k], rel=1e-4, abs=1e-7), k


def test_batched_ppo_with_depth_cameras(tmp_path):
    """rgbd_0/rgbd_1 + relative_image_timestamp through the Extractor's CNN branches
    (mlp_policy.py:25-46): rollout images stored, graph update over dict observations."""
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger, read_progress
    from ballbot_rl.training.ppo import BatchedPPO

    env = BallbotVecEnv(256, device="cuda:0", max_ep_steps=10, seed=5, disable_cameras=False)
    m = BatchedPPO(env, n_steps=8, batch_size=512, n_epochs=2, ent_coef=0.001, clip_range=0.015, vf_coef=2.0,
                   target_kl=0.3, learning_rate=1e-4, normalize_advantage=False, seed=10,
                   logger=CSVLogger(str(tmp_path), stdout=False))
    assert m.policy.features_extractor.features_dim == 15 + 1 + 20 + 20
    m.learn(total_timesteps=256 * 8 * 3)
    assert m._graphs is not None and "depth" in m._graphs.data
    assert float(m.buf.depth.min()) > 0 and float(m.buf.depth.max()) <= 1.0
    ts = m.buf.rel_ts.cpu().numpy()
    assert set(np.round(np.unique(ts) / 0.002).astype(int)) <= set(range(6))
    cols = read_progress(str(tmp_path / "progress.csv"))
    assert all(np.isfinite(x) for x in cols["train/loss"][1:])
    env.close()


@pytest.mark.parametrize("normalize", [False, True])
def test_fused_ppo_loss_matches_torch(normalize):
    """bb_ppo_loss (loss terms + gradients) vs the torch expression of SB3 PPO.train."""
    from ballbot_rl.training.ppo import _PPOLossHIP

    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(3)
    B = 8192
    mean = torch.randn(B, 3, generator=g).to(dev).requires_grad_()
    values = torch.randn(B, generator=g).to(dev).requires_grad_()
    log_std = (0.3 * torch.randn(3, generator=g)).to(dev).requires_grad_()
    actions = torch.randn(B, 3, generator=g).to(dev)
    adv = torch.randn(B, generator=g).to(dev)
    ret = torch.randn(B, generator=g).to(dev)
    with torch.no_grad():  # old log-probs: exact ties (rho = 1) on a third, far off on a third
        lp = torch.distributions.Normal(mean, torch.exp(log_std)).log_prob(actions).sum(-1)
        old = lp.clone()
        old[B // 3:2 * B // 3] += 0.5 * torch.randn(B // 3 + (2 * B // 3 - B // 3 - B // 3), generator=g).to(dev)
        old[2 * B // 3:] += 0.01 * torch.randn(B - 2 * B // 3, generator=g).to(dev)
    clip, ent_coef, vf_coef = 0.015, 0.001, 2.0

    def ref(mean, values, log_std):
        lp = torch.distributions.Normal(mean, torch.exp(log_std)).log_prob(actions).sum(-1)
        ent = torch.distributions.Normal(mean, torch.exp(log_std)).entropy().sum(-1)
        a = (adv - adv.mean()) / (adv.std() + 1e-8) if normalize else adv
        lr = lp - old
        r = torch.exp(lr)
        pg = -torch.min(a * r, a * torch.clamp(r, 1 - clip, 1 + clip)).mean()
        vf = torch.nn.functional.mse_loss(ret, values)
        el = -torch.mean(ent)
        return pg + ent_coef * el + vf_coef * vf, pg, vf, el, torch.mean((r - 1) - lr), \
            torch.mean((torch.abs(r - 1) > clip).float())

    lref, *tref = ref(mean, values, log_std)
    gref = torch.autograd.grad(lref, (mean, values, log_std))
    loss, t = _PPOLossHIP.apply(mean, values, log_std, actions, old, adv, ret, torch.tensor(clip, device=dev),
                                normalize, ent_coef, vf_coef)
    got = torch.autograd.grad(loss, (mean, values, log_std))
    assert torch.allclose(loss, lref, rtol=1e-5, atol=1e-6)
    for a, b in zip(t, tref):
        assert torch.allclose(a, b.float(), rtol=1e-4, atol=1e-6), (a, b)
    for a, b in zip(got, gref):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-7), (a - b).abs().max()


def test_encoder_pretrain_on_gpu_frames(tmp_path):
    """Depth frames straight from the GPU cameras -> TinyAutoencoder -> frozen encoder in PPO."""
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.encoders import TinyAutoencoder, collect_depth_images, load_frozen_encoder, train_autoencoder
    from ballbot_rl.training.ppo import BatchedPPO

    env = BallbotVecEnv(256, device="cuda:0", terrain_config={"type": "perlin", "config": {}}, n_terrains=4,
                        disable_cameras=False, seed=1)
    imgs = collect_depth_images(env, 4000, seed=1)
    assert imgs.shape == (4000, 1, 64, 64) and float(imgs.max()) <= 1.0 and float(imgs.min()) > 0
    path = str(tmp_path / "enc.safetensors")
    h = train_autoencoder(TinyAutoencoder(64, 64), imgs, epochs=3, batch_size=256, save_path=path,
                          log=lambda *_: None)
    assert h["best_val_loss"] < 0.05
    enc = load_frozen_encoder(path, device="cuda:0")
    m = BatchedPPO(env, n_steps=8, batch_size=512, n_epochs=1, learning_rate=1e-4, seed=2, frozen_encoder=enc)
    w0 = m.policy.features_extractor.extractors["rgbd_0"][0].weight.clone()
    m.learn(total_timesteps=256 * 8 * 2)
    assert torch.equal(w0, m.policy.features_extractor.extractors["rgbd_0"][0].weight)  # frozen
    env.close()


def test_split_k_linear_matches_linear():
    from ballbot_rl.policies.mlp_policy import SplitKLinear

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    lin = SplitKLinear(128, 128).to(dev)
    ref = torch.nn.Linear(128, 128).to(dev)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(8192, 128, device=dev, requires_grad=True)
    x2 = x.detach().clone().requires_grad_()
    gy = torch.randn(8192, 128, device=dev)
    lin(x).backward(gy)
    ref(x2).backward(gy)
    assert torch.allclose(x.grad, x2.grad, rtol=1e-5, atol=1e-5)
    assert torch.allclose(lin.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)
    assert torch.allclose(lin.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("max_norm", [0.5, 1e3])
def test_flat_adamw_matches_torch(max_norm):
    """bb_adamw_clip (FlatAdamW) vs clip_grad_norm_ + torch.optim.AdamW over several steps
    with a changing learning rate; max_norm 0.5 clips every step, 1e3 never."""
    from ballbot_rl.training.optim import FlatAdamW

    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    shapes = [(128, 15), (128,), (128, 128), (128,), (3, 128), (3,), (3,)]
    ref = [torch.nn.Parameter(torch.randn(s, device=dev) * 0.1) for s in shapes]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    opt_ref = torch.optim.AdamW(ref, lr=3e-4, weight_decay=0.01)
    opt = FlatAdamW(mine, lr=3e-4, weight_decay=0.01, max_grad_norm=max_norm)
    assert all(p.data_ptr() >= opt.flat.data_ptr() for p in mine)  # views of the flat buffer
    for step in range(6):
        lr = 3e-4 * (1 - step / 10)
        opt_ref.param_groups[0]["lr"] = lr
        opt.param_groups[0]["lr"].fill_(lr)
        grads = [torch.randn(s, device=dev) for s in shapes]
        for p, q, g in zip(ref, mine, grads):
            p.grad = g.clone()
            q.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt_ref.step()
        opt.step()
    torch.cuda.synchronize()
    assert float(opt.step_t) == 6.0
    for p, q in zip(ref, mine):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-7), (p - q).abs().max()
    for p, q in zip(ref, mine):
        st = opt_ref.state[p]
        # m = 0.9 m + 0.1 g cancels for small m: an fma contraction moves it by ~ulp(0.1 |g|)
        assert torch.allclose(st["exp_avg"], opt.state[q]["exp_avg"], rtol=1e-5, atol=1e-7), \
            (st["exp_avg"] - opt.state[q]["exp_avg"]).abs().max()
        assert torch.allclose(st["exp_avg_sq"], opt.state[q]["exp_avg_sq"], rtol=1e-5, atol=1e-9), \
            (st["exp_avg_sq"] - opt.state[q]["exp_avg_sq"]).abs().max()


def test_adamw_clip_rejects_bad_arguments():
    from ballbot_gym import _native as N

    L = N.lib()
    x = torch.zeros(16, device="cuda:0")
    s = torch.zeros(4, device="cuda:0")
    p = x.data_ptr()
    assert L.bb_adamw_clip(p, p, p, p, 0, p, s.data_ptr(), s.data_ptr(), 0.9, 0.999, 1e-8, 0.01, 0.5, None) < 0
    assert "n must be" in N.last_error()
    assert L.bb_adamw_clip(p, p, p, p, 16, p, s.data_ptr(), s.data_ptr(), 1.0, 0.999, 1e-8, 0.01, 0.5, None) < 0
    assert L.bb_adamw_clip(None, p, p, p, 16, p, s.data_ptr(), s.data_ptr(), 0.9, 0.999, 1e-8, 0.01, 0.5, None) < 0



def _gpu_fake(n=256, ep_len=6):
    from fake_env import FakeEnv

    dev = torch.device("cuda:0")

    class GpuFake(FakeEnv):
        def __init__(self):
            super().__init__(n, ep_len=ep_len)
            self.device = dev

        def reset(self):
            o, i = super().reset()
            return o.to(dev), i

        def step(self, a):
            o, r, d, t, i = super().step(a.cpu())
            return o.to(dev), r.to(dev), d.to(dev), t.to(dev), i

    return GpuFake()


def _sb3_minibatch_loss(policy, obs, act, old_logp, adv, ret, clip, ent_coef, vf_coef, normalize):
    """SB3 2.6.0 PPO.train's minibatch loss in plain torch autograd (the checker)."""
    values, logp, entropy = policy.evaluate_actions(obs, act)
    if normalize:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    lr = logp - old_logp
    r = torch.exp(lr)
    pg = -torch.min(adv * r, adv * torch.clamp(r, 1 - clip, 1 + clip)).mean()
    vf = torch.nn.functional.mse_loss(ret, values)
    ent = -torch.mean(entropy)
    with torch.no_grad():
        kl = torch.mean((r - 1) - lr)
        cf = torch.mean((torch.abs(r - 1) > clip).float())
    return pg + ent_coef * ent + vf_coef * vf, pg, vf, ent, kl, cf


@pytest.mark.parametrize("normalize", [True, False])
def test_fused_minibatch_matches_autograd(normalize):
    """bb_ppo_mlp_step (one graph replay = one minibatch): gradients and log terms
    vs torch autograd of the SB3 loss on the same parameters and samples (fp32;
    only summation orders differ), and the AdamW step it applies vs FlatAdamW on
    the autograd gradients."""
    import copy

    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.optim import FlatAdamW
    from ballbot_rl.training.ppo import BatchedPPO, _UpdateGraphs

    m = BatchedPPO(_gpu_fake(), n_steps=16, batch_size=512, n_epochs=2, learning_rate=1e-3, clip_range=0.1,
                   ent_coef=0.01, vf_coef=0.5, normalize_advantage=normalize, seed=5,
                   logger=CSVLogger(None, stdout=False))
    m.collect_rollouts()
    with torch.no_grad():  # spread the log ratio over the clip range
        m.buf.log_probs.add_(0.1 * torch.randn_like(m.buf.log_probs))
    d = {k: v.clone() for k, v in m.buf.flat().items()}
    n = d["obs"].shape[0]
    gr = _UpdateGraphs(m, n)
    assert gr.fused
    for k, v in gr.data.items():
        v.copy_(d[k])
    gr.clip.fill_(0.1)
    perm = torch.randperm(n, device=m.device).view(gr.nb, -1)
    gr.perm.copy_(perm)
    gr.k.fill_(3); gr.row.zero_()
    ref_policy = copy.deepcopy(m.policy)
    ref_params = [p for p in ref_policy.parameters()]
    gr.graph.replay()
    torch.cuda.synchronize()
    assert int(gr.k) == 4 and int(gr.row) == 1
    idx = perm[3]
    loss, pg, vf, ent, kl, cf = _sb3_minibatch_loss(ref_policy, d["obs"][idx], d["actions"][idx], d["log_probs"][idx],
                                                    d["advantages"][idx], d["returns"][idx], 0.1, 0.01, 0.5, normalize)
    loss.backward()
    row = gr.log[0]
    for got, want in zip(row.tolist(), (loss, pg, vf, ent, kl, cf)):
        assert got == pytest.approx(float(want.detach()), rel=2e-4, abs=1e-6)
    opt = m.optimizer
    names = [nm for nm, _ in m.policy.named_parameters()]
    where = {id(p): o for p, o in zip(opt.params, opt.offsets)}
    for nm, p, q in zip(names, m.policy.parameters(), ref_params):
        off = where[id(p)]
        g = opt.grad[off:off + p.numel()].view_as(p)
        scale = float(q.grad.abs().max())
        err = float((g - q.grad).abs().max())
        assert err <= 2e-4 * scale + 1e-8, (nm, err, scale)
    # the AdamW step taken: FlatAdamW (tested against torch) on the autograd gradients
    ref_opt = FlatAdamW(ref_params, lr=float(opt.lr), weight_decay=opt.weight_decay, max_grad_norm=opt.max_grad_norm)
    ref_opt.step()
    for p, q in zip(m.policy.parameters(), ref_params):
        diff = (p.detach() - q.detach()).abs()
        # first Adam step ~ lr * sign(g): elements whose gradient is ~0 may flip
        assert float((diff > 1e-6).float().mean()) < 2e-3, float(diff.max())
        assert float(diff.max()) <= 2.5e-3


@pytest.mark.parametrize("target_kl", [None, 2e-3])
def test_fused_update_matches_autograd_update(target_kl, monkeypatch):
    """A whole update (all epochs, device-side KL stop) with the fused minibatch
    vs the autograd graphs: same number of updates, log terms and parameters
    within the fp32 reduction-order tolerance."""
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    models = []
    for _ in range(2):
        m = BatchedPPO(_gpu_fake(), n_steps=16, batch_size=512, n_epochs=3, learning_rate=3e-4, target_kl=target_kl,
                       normalize_advantage=True, seed=4, logger=CSVLogger(None, stdout=False))
        m.collect_rollouts()
        models.append(m)
    d0 = models[0].buf.flat()
    for fused, m in zip(("0", "1"), models):  # the update graphs are built (and the path chosen) in _update
        monkeypatch.setenv("BB_PPO_FUSED", fused)
        m.shuffle_gen.manual_seed(99)
        m._update({k: v.clone() for k, v in d0.items()})
    assert not models[0]._graphs.fused and models[1]._graphs.fused
    assert models[0]._n_updates == models[1]._n_updates
    la, lb = models[0].logger.values, models[1].logger.values
    for k in ("train/policy_gradient_loss", "train/value_loss", "train/approx_kl", "train/clip_fraction"):
        assert la[k] == pytest.approx(lb[k], rel=5e-3, abs=1e-6), k
    for a, b in zip(models[0].policy.parameters(), models[1].policy.parameters()):
        diff = (a - b).abs()
        assert float((diff > 1e-5).float().mean()) < 1e-2, float(diff.max())


def test_ppo_mlp_step_rejects_bad_arguments():
    import ctypes as C

    from ballbot_gym import _native as N

    L = N.lib()
    nb = C.c_int64()
    assert L.bb_ppo_mlp_workspace_bytes(100, C.byref(nb)) < 0
    assert L.bb_ppo_mlp_workspace_bytes(8192, C.byref(nb)) == 0 and nb.value > 8192 * 2000 * 4
    a = N.PPOMlpArgs()
    assert L.bb_ppo_mlp_step(C.byref(a), None) < 0
    assert "NULL" in N.last_error()


def test_fused_rollout_matches_torch(monkeypatch):
    """collect_rollouts with bb_ppo_mlp_act + bb_rollout_track vs the torch loop:
    same noise, same env stream -> the same buffers (fp32 reduction-order
    tolerance for the network outputs) and the same finished episodes."""
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    models = []
    for fused in ("0", "1"):
        monkeypatch.setenv("BB_PPO_FUSED", fused)
        m = BatchedPPO(_gpu_fake(n=300, ep_len=5), n_steps=12, batch_size=256, n_epochs=1, seed=7,
                       logger=CSVLogger(None, stdout=False))
        for _ in range(2):
            m.collect_rollouts()
        models.append(m)
    assert models[0]._act_slots is False and models[1]._act_slots
    a, b = models[0].buf, models[1].buf
    assert torch.equal(a.obs, b.obs) and torch.equal(a.starts, b.starts)
    assert torch.allclose(a.actions, b.actions, rtol=1e-5, atol=1e-5), (a.actions - b.actions).abs().max()
    assert torch.allclose(a.values, b.values, rtol=1e-4, atol=1e-5), (a.values - b.values).abs().max()
    assert torch.allclose(a.log_probs, b.log_probs, rtol=1e-4, atol=1e-4), (a.log_probs - b.log_probs).abs().max()
    assert torch.allclose(a.rewards, b.rewards, rtol=1e-4, atol=1e-5)
    assert torch.allclose(a.advantages, b.advantages, rtol=1e-3, atol=1e-4)
    ea, eb = list(models[0].ep_info_buffer), list(models[1].ep_info_buffer)
    assert len(ea) == len(eb) > 0
    assert [e["l"] for e in ea] == [e["l"] for e in eb]
    assert np.allclose([e["r"] for e in ea], [e["r"] for e in eb], rtol=1e-4, atol=1e-4)
    assert models[0].num_timesteps == models[1].num_timesteps


def test_fused_act_deterministic_is_the_mean():
    """bb_ppo_mlp_act with noise NULL: actions = the policy mean (predict(deterministic=True) before the clip)."""
    import ctypes as C

    from ballbot_gym import _native as N
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO, fused_mlp_slots

    m = BatchedPPO(_gpu_fake(n=100), n_steps=4, batch_size=256, seed=2, logger=CSVLogger(None, stdout=False))
    slots = fused_mlp_slots(m, update=False)
    assert slots is not None
    dev = m.device
    obs = torch.randn(77, 15, device=dev)
    act = torch.empty(77, 3, device=dev); val = torch.empty(77, device=dev); lp = torch.empty(77, device=dev)
    clipped = torch.empty(77, 3, device=dev)
    ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    N.check(N.lib().bb_ppo_mlp_act(ptr(m.optimizer.flat), (C.c_int32 * 21)(*slots), m.optimizer.flat.numel(), ptr(obs),
                                   15, None, 77, None, ptr(act), ptr(clipped), ptr(val), ptr(lp), None),
            "bb_ppo_mlp_act")
    torch.cuda.synchronize()
    with torch.no_grad():
        mean, v = m.policy._heads(obs)
        want_lp = m.policy.log_prob(mean, mean)
    assert torch.allclose(act, mean, rtol=1e-5, atol=1e-6)
    assert torch.equal(clipped, act.clamp(-1, 1))
    assert torch.allclose(val, v, rtol=1e-5, atol=1e-5)
    assert torch.allclose(lp, want_lp, rtol=1e-6, atol=1e-5)


def _random_frozen_encoder(seed=0):
    from ballbot_rl.encoders import TinyAutoencoder

    g = torch.Generator().manual_seed(seed)
    enc = TinyAutoencoder(64, 64).encoder
    with torch.no_grad():
        for mod in enc:
            if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
                nf = mod.num_features
                mod.weight.copy_(1 + 0.2 * torch.randn(nf, generator=g))
                mod.bias.copy_(0.1 * torch.randn(nf, generator=g))
                mod.running_mean.copy_(0.1 * torch.randn(nf, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(nf, generator=g))
    for p in enc.parameters():
        p.requires_grad = False
    return enc.to("cuda:0")


@pytest.mark.parametrize("train", [False, True])
def test_fused_encoder_matches_torch(train):
    """bb_depth_encoder vs the torch module (MIOpen convolutions) on a strided camera
    slice: features, and in train mode the running statistics and counters torch's
    BatchNorm updates (fp32; reduction orders differ)."""
    import copy

    from ballbot_rl.encoders.models import fusable_encoder, fused_encoder_forward

    ref = _random_frozen_encoder(3)
    mine = copy.deepcopy(ref)
    assert fusable_encoder(mine)
    ref.train(train); mine.train(train)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    cams = torch.rand(300, 2, 64, 64, device="cuda:0", generator=g) * 1.0
    for cam in (0, 1):
        x = cams[:, cam:cam + 1]
        with torch.no_grad():
            want = ref(x)
        got = fused_encoder_forward(mine, x)
        torch.cuda.synchronize()
        assert got.shape == (300, 20)
        assert torch.allclose(got, want, rtol=1e-4, atol=2e-4), (got - want).abs().max()
    for a, b in zip(ref.modules(), mine.modules()):
        if isinstance(a, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            assert torch.allclose(a.running_mean, b.running_mean, rtol=1e-4, atol=1e-5)
            assert torch.allclose(a.running_var, b.running_var, rtol=1e-4, atol=1e-5)
            assert int(a.num_batches_tracked) == int(b.num_batches_tracked) == (2 if train else 0)


def test_fused_encoder_in_extractor(monkeypatch):
    """The camera policy's Extractor with a frozen encoder: fused vs BB_FUSED_ENCODER=0."""
    from ballbot_rl.policies.mlp_policy import ActorCriticPolicy, obs_spaces

    enc = _random_frozen_encoder(4)
    pol = ActorCriticPolicy(obs_spaces(cameras=True), frozen_encoder=enc).to("cuda:0")
    assert pol.features_extractor._frozen_keys == {"rgbd_0", "rgbd_1"}
    n = 256
    obs = {k: torch.randn(n, 3, device="cuda:0") for k in ("actions", "angular_vel", "motor_state", "orientation",
                                                            "vel")}
    cams = torch.rand(n, 2, 64, 64, device="cuda:0")
    obs["rgbd_0"], obs["rgbd_1"] = cams[:, 0:1], cams[:, 1:2]
    obs["relative_image_timestamp"] = torch.rand(n, 1, device="cuda:0") * 0.01
    pol.eval()
    with torch.no_grad():
        fused = pol.features_extractor(obs)
        monkeypatch.setenv("BB_FUSED_ENCODER", "0")
        plain = pol.features_extractor(obs)
    assert torch.allclose(fused, plain, rtol=1e-4, atol=2e-4), (fused - plain).abs().max()


def test_fused_camera_policy_matches_autograd(monkeypatch):
    """The camera policy with fused frozen encoders: the fused minibatch over the 56-d
    features (bb_ppo_mlp_step, obs_direct) vs the autograd minibatch on the same
    rollout, and the fused rollout step vs the torch one on the first env step."""
    import copy

    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    enc = _random_frozen_encoder(5)
    envs = [BallbotVecEnv(256, device="cuda:0", seed=5, disable_cameras=False) for _ in range(2)]
    models = []
    for fused, env in zip(("0", "1"), envs):
        monkeypatch.setenv("BB_PPO_FUSED", fused)
        m = BatchedPPO(env, n_steps=8, batch_size=512, n_epochs=2, learning_rate=3e-4, seed=3,
                       frozen_encoder=copy.deepcopy(enc), logger=CSVLogger(None, stdout=False))
        m.collect_rollouts()
        models.append(m)
    assert models[0]._act_slots is False and models[1]._act_slots
    a, b = models[0].buf, models[1].buf
    assert torch.equal(a.obs[0], b.obs[0]) and torch.equal(a.depth[0], b.depth[0])
    assert torch.allclose(a.actions[0], b.actions[0], rtol=1e-4, atol=1e-5), (a.actions[0] - b.actions[0]).abs().max()
    assert torch.allclose(a.values[0], b.values[0], rtol=1e-4, atol=1e-5)
    assert torch.allclose(a.log_probs[0], b.log_probs[0], rtol=1e-4, atol=1e-4)
    d0 = models[0].buf.flat()
    for fused, m in zip(("0", "1"), models):
        monkeypatch.setenv("BB_PPO_FUSED", fused)
        m.shuffle_gen.manual_seed(99)
        m._update({k: v.clone() for k, v in d0.items()})
    assert not models[0]._graphs.fused and models[1]._graphs.fused
    la, lb = models[0].logger.values, models[1].logger.values
    for k in ("train/policy_gradient_loss", "train/value_loss", "train/approx_kl"):
        assert la[k] == pytest.approx(lb[k], rel=5e-3, abs=1e-6), k
    for p, q in zip(models[0].policy.parameters(), models[1].policy.parameters()):
        diff = (p - q).abs()
        assert float((diff > 1e-5).float().mean()) < 1e-2, float(diff.max())
    for p, q in zip(models[0].policy.features_extractor.buffers(), models[1].policy.features_extractor.buffers()):
        assert torch.allclose(p.double(), q.double(), rtol=1e-4, atol=1e-5)
    for env in envs:
        env.close()


def test_fused_encoder_index_gather():
    """bb_depth_encoder reading a minibatch through an index == encoding the gathered images."""
    import copy

    from ballbot_rl.encoders.models import fused_encoder_forward

    enc = _random_frozen_encoder(6)
    enc2 = copy.deepcopy(enc)
    enc.train(); enc2.train()
    cams = torch.rand(700, 2, 64, 64, device="cuda:0")
    idx = torch.randperm(700, device="cuda:0")[:512]
    a = fused_encoder_forward(enc, cams[:, 1:2], index=idx)
    b = fused_encoder_forward(enc2, cams[idx][:, 1:2].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    for p, q in zip(enc.buffers(), enc2.buffers()):
        assert torch.equal(p, q)


def test_camera_feature_cache_is_exact(monkeypatch):
    """The camera rollout re-encodes only the envs whose cameras re-rendered this step
    (relative_image_timestamp 0); the rollout buffers equal a full re-encode every step."""
    import copy

    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    enc = _random_frozen_encoder(7)
    bufs = []
    for cache in ("1", "0"):
        monkeypatch.setenv("BB_ENC_CACHE", cache)
        env = BallbotVecEnv(256, device="cuda:0", seed=9, disable_cameras=False, max_ep_steps=5)
        m = BatchedPPO(env, n_steps=14, batch_size=512, seed=3, frozen_encoder=copy.deepcopy(enc),
                       logger=CSVLogger(None, stdout=False))
        m.collect_rollouts()
        assert m._act_slots
        bufs.append((m.buf.actions.clone(), m.buf.values.clone(), m.buf.rel_ts.clone()))
        env.close()
    (a0, v0, r0), (a1, v1, r1) = bufs
    assert float((r0 == 0).float().mean()) < 0.5  # most steps reuse cached features
    assert torch.equal(r0, r1) and torch.equal(a0, a1) and torch.equal(v0, v1)


def test_rollout_graph_matches_eager(monkeypatch):
    """The proprio rollout captured as ONE HIP graph (n_steps x [policy step, bb_step with the
    two-stream route, bookkeeping]) replays bit-identically to the eager fused rollout -- the
    same noise, the same env stream -- also after the caching allocator has been churned and
    emptied between replays (every pointer the graph holds is a fixed buffer, _RolloutGraph)."""
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    monkeypatch.setenv("BB_FUSED_ROLLOUT", "0")  # the per-step rollout (bb_rollout is tested in test_gpu_rollout.py)
    models = []
    for graph in ("0", "1"):
        monkeypatch.setenv("BB_ROLLOUT_GRAPH", graph)
        env = BallbotVecEnv(512, device="cuda:0", seed=6, terrain_config={"type": "perlin", "config": {}},
                            n_terrains=8)  # relief bank: the predict/split route on two streams
        m = BatchedPPO(env, n_steps=16, batch_size=1024, n_epochs=1, seed=4, logger=CSVLogger(None, stdout=False))
        bufs = []
        for r in range(3):
            m.collect_rollouts()
            bufs.append({k: getattr(m.buf, k).clone() for k in ("obs", "actions", "values", "log_probs", "rewards",
                                                                 "starts", "advantages", "returns")})
            junk = [torch.empty(1 << 24, device="cuda:0") for _ in range(8)]  # allocator churn
            del junk
            torch.cuda.empty_cache()
        models.append((m, bufs, env))
    (ma, ba, ea), (mb, bb, eb) = models
    assert ma._rgraph is None and mb._rgraph is not None
    for r in range(3):
        for k in ba[r]:
            assert torch.equal(ba[r][k], bb[r][k]), (r, k)
    assert [e["r"] for e in ma.ep_info_buffer] == [e["r"] for e in mb.ep_info_buffer]
    assert [e["l"] for e in ma.ep_info_buffer] == [e["l"] for e in mb.ep_info_buffer]
    qa, va, _, sa = ea.get_state()
    qb, vb, _, sb = eb.get_state()
    assert np.array_equal(qa, qb) and np.array_equal(va, vb) and np.array_equal(sa, sb)
    ea.close()
    eb.close()


def test_update_graph_build_keeps_encoder_statistics(monkeypatch):
    """Building the update graphs runs warm-up minibatches in train mode on a zero buffer:
    the frozen encoders' BatchNorm running statistics and num_batches_tracked must be
    exactly as before the build."""
    import copy

    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    env = BallbotVecEnv(256, device="cuda:0", seed=5, disable_cameras=False)
    m = BatchedPPO(env, n_steps=8, batch_size=512, n_epochs=1, seed=3, frozen_encoder=copy.deepcopy(
        _random_frozen_encoder(7)), logger=CSVLogger(None, stdout=False))
    m.collect_rollouts()
    before = [b.clone() for b in m.policy.buffers()]
    assert len(before) > 0
    m._graphs_for(256 * 8)
    for b0, b1 in zip(before, m.policy.buffers()):
        assert torch.equal(b0, b1)
    env.close()


def _dp_gpu_worker(rank, world, port, q, mode="allreduce"):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)  # two ranks sharing the box's GPU
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    torch.manual_seed(10 + rank)
    env = BallbotVecEnv(256, device="cuda:0", seed=3 + rank, max_ep_steps=40)
    m = BatchedPPO(env, n_steps=16, batch_size=1024, n_epochs=2, seed=5, update_mode=mode,
                   logger=CSVLogger(None, stdout=False))
    m.warm_up()
    m.learn(total_timesteps=256 * 16 * world * 2)
    vec = torch.nn.utils.parameters_to_vector(m.policy.parameters()).detach().cpu()
    q.put((rank, vec.numpy(), m._n_updates, float(m.logger.values.get("train/value_loss", float("nan")))))
    env.close()
    dist.destroy_process_group()


def test_data_parallel_update_on_gpu_ranks():
    """update_mode="allreduce" with the GPU env, bb_ppo_loss and FlatAdamW (bb_adamw_clip) on
    two ranks (gloo, one GPU): different env shards, the same parameters after every update."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, v0, u0, l0), (_, v1, u1, l1) = res
    assert (v0 == v1).all() and u0 == u1 == 4 and l0 == l1 and np.isfinite(l0)


def test_gather_update_on_gpu_ranks():
    """The multi-rank default, update_mode="gather", with the GPU env on two ranks sharing the GPU
    over gloo: the rollouts (device buffers; gloo gathers them through host memory) reach rank 0,
    which updates and broadcasts -- both ranks end with the same parameters, rank 0 counts the
    epochs.  warm_up() builds rank 0's update graphs for the gathered size before learn()."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_gpu_worker, args=(r, 2, port, q, "gather")) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, v0, u0, l0), (_, v1, u1, l1) = res
    assert (v0 == v1).all() and u0 == 4 and u1 == 0 and np.isfinite(l0)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_data_parallel_update_graph_on_one_rank(fused, monkeypatch):
    """update_mode="allreduce" through the captured update graphs (the form RCCL ranks run: the
    global advantage statistics and the gradient all-reduce are graph nodes; the fused minibatch
    splits around them, bb_ppo_mlp_args.phase 1 / 2 with adv_stats).  At world size 1 the
    collectives are the identity, so the graph must equal the eager data-parallel loop, and the
    split fused minibatch the unsplit one, to the fp32 reduction-order tolerance.  The RCCL
    capture itself needs a multi-GPU node: unmeasured on hardware."""
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    monkeypatch.setenv("BB_PPO_FUSED", fused)
    models = []
    for dp, graphs in ((True, True), (True, False), (False, True)):
        m = BatchedPPO(_gpu_fake(), n_steps=16, batch_size=512, n_epochs=3, learning_rate=3e-4, target_kl=None,
                       normalize_advantage=True, seed=4, use_graphs=graphs, update_mode="allreduce",
                       logger=CSVLogger(None, stdout=False))
        m._force_dp = dp
        m.collect_rollouts()
        models.append(m)
    d0 = models[0].buf.flat()
    for m in models:
        m.shuffle_gen.manual_seed(99)
        m._update({k: v.clone() for k, v in d0.items()}, dp=m._dp)
    g = models[0]._graphs
    assert g is not None and g.dp and g.fused == (fused == "1") and models[1]._graphs is None
    assert models[0]._n_updates == models[1]._n_updates == models[2]._n_updates == 3
    for ref in models[1:]:
        la, lb = models[0].logger.values, ref.logger.values
        for k in ("train/policy_gradient_loss", "train/value_loss", "train/approx_kl", "train/clip_fraction"):
            assert la[k] == pytest.approx(lb[k], rel=5e-3, abs=1e-6), k
        for a, b in zip(models[0].policy.parameters(), ref.policy.parameters()):
            diff = (a - b).abs()
            assert float((diff > 1e-5).float().mean()) < 1e-2, float(diff.max())


@pytest.mark.parametrize("terrain", ["flat", "perlin", "cameras"])
def test_warm_up_keeps_the_trajectory(terrain):
    """BatchedPPO.warm_up (update graphs captured and primed on zero data, BLAS initialised) before
    learn() leaves the training trajectory as it was: the same parameters and logs after three
    iterations as a trainer that builds its graphs inside its first update."""
    import copy

    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    cams = terrain == "cameras"  # the camera policy with a frozen encoder: BatchNorm statistics restored too
    kw = {"n_terrains": None} if terrain == "perlin" else {}
    enc = _random_frozen_encoder(7) if cams else None  # ONE encoder (its conv weights come from torch's RNG)
    res = []
    for warm in (False, True):
        env = BallbotVecEnv(512, device="cuda:0", seed=21, disable_cameras=not cams,
                            terrain_config={"type": "flat" if cams else terrain, "config": {}}, **kw)
        extra = {"frozen_encoder": copy.deepcopy(enc)} if cams else {}
        m = BatchedPPO(env, n_steps=16, batch_size=2048, n_epochs=2, ent_coef=0.001, clip_range=0.015, vf_coef=2.0,
                       target_kl=0.3, seed=6, logger=CSVLogger(None, stdout=False), **extra)
        if warm:
            m.warm_up()
            assert m._graphs is not None and m._graphs.fused
        m.learn(total_timesteps=512 * 16 * 3)
        vec = torch.nn.utils.parameters_to_vector(m.policy.parameters()).detach().cpu().numpy()
        bufs = [b.detach().cpu().numpy().astype(np.float64).ravel() for b in m.policy.buffers()]
        res.append((vec, dict(m.logger.values), m._n_updates, len(m.ep_info_buffer), bufs))
        env.close()
    (v0, l0, u0, e0, b0), (v1, l1, u1, e1, b1) = res
    for x, y in zip(b0, b1):  # BatchNorm running statistics of the frozen encoders (cameras)
        np.testing.assert_allclose(x, y, rtol=0, atol=1e-6)
    assert u0 == u1 == 6 and e0 == e1
    np.testing.assert_allclose(v0, v1, rtol=0, atol=1e-6)
    for k in ("train/value_loss", "train/policy_gradient_loss", "train/approx_kl"):
        assert l0[k] == pytest.approx(l1[k], rel=1e-5, abs=1e-8), k
