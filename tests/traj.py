"""Oracle trajectory recorder for teacher-forced parity tests (test helper)."""
import numpy as np

import oracle_lib as O


def record(n_envs, n_steps, hfield, size_z=2.0, seed=0, action_scale=1.0, max_ep_steps=4000, pid_frac=0.5):
    """Run n_envs oracle envs for n_steps with random (and PID) actions.

    Returns dict of arrays indexed [t, env]: qpos/qvel/warm/steps before the
    step, the action, and the oracle's post-step state, obs, reward, flags.
    Terminated envs are reset (with the terrain's init offset) before the
    next recorded step, so every record is a valid teacher-forced pair."""
    from pid_ref import PID, rotvec_to_R

    rng = np.random.default_rng(seed)
    cfg = O.default_cfg(max_ep_steps=max_ep_steps)
    off = O.init_offset(hfield, size_z)
    st = [O.reset_state(off) for _ in range(n_envs)]
    sc = [np.zeros(1, np.int32) for _ in range(n_envs)]
    pids = [PID(0.002, 20, 15, 2) for _ in range(n_envs)]
    use_pid = rng.random(n_envs) < pid_frac
    last_obs = [np.zeros(15, np.float32) for _ in range(n_envs)]
    out = {k: [] for k in ("qpos", "qvel", "warm", "steps", "action", "qpos1", "qvel1", "warm1", "obs", "reward",
                           "flags", "pos2d")}
    for t in range(n_steps):
        rows = {k: [] for k in out}
        for e in range(n_envs):
            q, v, w = st[e]
            rows["qpos"].append(q.copy()); rows["qvel"].append(v.copy()); rows["warm"].append(w.copy())
            rows["steps"].append(int(sc[e][0]))
            if use_pid[e]:
                a = pids[e].act(rotvec_to_R(last_obs[e][9:12])) + rng.normal(0, 0.3, 3)
                a = np.clip(a, -1.5, 1.5).astype(np.float32)
            else:
                a = (rng.uniform(-1, 1, 3) * action_scale).astype(np.float32)
            rows["action"].append(a)
            obs, r, fl, p2, _ = O.env_step(cfg, q, v, w, sc[e], a, hfield, size_z)
            rows["qpos1"].append(q.copy()); rows["qvel1"].append(v.copy()); rows["warm1"].append(w.copy())
            rows["obs"].append(obs); rows["reward"].append(r); rows["flags"].append(fl); rows["pos2d"].append(p2)
            last_obs[e] = obs
            if fl & 1:
                st[e] = O.reset_state(off)
                sc[e][:] = 0
                pids[e] = PID(0.002, 20, 15, 2)
                last_obs[e] = np.zeros(15, np.float32)
        for k in out:
            out[k].append(np.array(rows[k]))
    return {k: np.array(v) for k, v in out.items()}
