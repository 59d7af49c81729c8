"""VecNormalize across ranks (world size 2, gloo, CPU): SB3 keeps ONE RunningMeanStd over all envs of
the VecEnv, so a 2-rank run over shards of 6 envs must end with the same obs_rms / ret_rms and the same
normalised outputs as a 1-rank run over all 12 envs.  The device kernels are replaced (test only) by the
numpy restatement of SB3's VecNormalize (oracle/vecnorm_ref.py); what this checks is the host logic
around them: the packed all-gather in global env-id order, the statistics sized for the global batch
and each rank's slice of the outputs."""
import os
import socket
from types import SimpleNamespace

import numpy as np
import torch
import torch.multiprocessing as mp

N_LOCAL, DIM, STEPS = 6, 5, 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class ShardEnv:
    """Deterministic per-global-env outputs; episode ends every 3 steps for odd global ids."""

    def __init__(self, n, offset):
        self.num_envs, self.offset, self.t = n, offset, 0
        self.observation_space = SimpleNamespace(shape=(DIM,))
        self.action_space = SimpleNamespace(low=np.zeros(1), high=np.ones(1))
        self.stepper = SimpleNamespace(device="cpu", reset=self._reset)

    def _rows(self, t):
        gid = np.arange(self.offset, self.offset + self.num_envs)[:, None]
        return np.sin(0.37 * gid + 1.3 * t + np.arange(DIM)[None, :]) * (1 + 0.1 * gid)

    def _reset(self):
        self.t = 0
        return torch.from_numpy(self._rows(0))

    def step_torch(self, actions):
        self.t += 1
        gid = np.arange(self.offset, self.offset + self.num_envs)
        obs = torch.from_numpy(self._rows(self.t))
        rew = torch.from_numpy(np.cos(0.5 * gid + self.t))
        done = ((gid % 2 == 1) & (self.t % 3 == 0)).astype(np.uint8)
        term = torch.from_numpy(done)
        trunc = torch.zeros_like(term)
        tobs = torch.from_numpy(self._rows(self.t + 100))
        return obs, rew, term, trunc, tobs


def _cpu_vecnormalize(**kw):
    """VecNormalize with its two kernels restated in numpy (SB3 order), state kept in its tensors."""
    from oracle.vecnorm_ref import VecNormalizeRef
    from ur3e_amd.envs.vec_normalize import VecNormalize

    class CpuVN(VecNormalize):
        def _stream(self):
            return None

        def _sync_from(self, ref):
            self._obs_mean.copy_(torch.from_numpy(np.asarray(ref.obs_rms.mean, dtype=np.float64)))
            self._obs_var.copy_(torch.from_numpy(np.asarray(ref.obs_rms.var, dtype=np.float64)))
            self._obs_count.fill_(float(ref.obs_rms.count))
            self._ret_mean.fill_(float(ref.ret_rms.mean))
            self._ret_var.fill_(float(ref.ret_rms.var))
            self._ret_count.fill_(float(ref.ret_rms.count))
            self._returns.copy_(torch.from_numpy(ref.returns))

        def _kernel_reset(self, n, obs, obs_out):
            assert n == self.n_stats and obs.shape == (n, self.dim)
            self.ref = VecNormalizeRef(n, self.dim, norm_reward=self.norm_reward)
            obs_out.copy_(torch.from_numpy(self.ref.reset(obs.numpy())))
            self._sync_from(self.ref)

        def _kernel_step(self, n, obs, rew, term, trunc, tobs):
            assert n == self.n_stats
            dones = (term.numpy() | trunc.numpy()).astype(bool)
            out, r, t = self.ref.step(obs.numpy(), rew.numpy(), dones, tobs.numpy())
            self._obs_out.copy_(torch.from_numpy(out))
            self._rew_out.copy_(torch.from_numpy(np.asarray(r, dtype=np.float64)))
            for i, row in t.items():
                self._tobs_out[i] = torch.from_numpy(row)
            self._sync_from(self.ref)

    return CpuVN(**kw)


def _run(rank, world, group, out_path):
    env = ShardEnv(N_LOCAL * (2 // world), rank * N_LOCAL)
    vn = _cpu_vecnormalize(venv=env, norm_reward=True, group=group)
    rows = [vn.reset_torch().numpy().copy()]
    for _ in range(STEPS):
        o, r, term, trunc, to = vn.step_torch(None)
        rows.append(np.concatenate([o.numpy(), r.numpy()[:, None], to.numpy()], 1))
    stats = np.concatenate([vn.obs_rms.mean, vn.obs_rms.var, [vn.obs_rms.count], vn.ret_rms.mean.ravel(),
                            vn.ret_rms.var.ravel(), [vn.ret_rms.count], vn.returns])
    np.save(out_path, np.concatenate([np.concatenate(rows[1:], 0).ravel(), rows[0].ravel(), stats]))


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _run(rank, world, dist.group.WORLD, out_path + f".r{rank}.npy")
    dist.destroy_process_group()


def test_vecnormalize_two_ranks_match_one(tmp_path):
    one = str(tmp_path / "one.npy")
    _run(0, 1, None, one)
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path / "two")), nprocs=2, join=True)
    a = np.load(one)
    r0 = np.load(str(tmp_path / "two.r0.npy"))
    r1 = np.load(str(tmp_path / "two.r1.npy"))
    # rank 0 owns global envs 0..5, rank 1 owns 6..11: reassemble per step and compare everything
    width = DIM + 1 + DIM
    n_rows = STEPS * N_LOCAL * width
    nst = 2 * DIM + 1 + 1 + 1 + 1
    s1, s0, sa = r1[-(nst + N_LOCAL):], r0[-(nst + N_LOCAL):], a[-(nst + 2 * N_LOCAL):]
    # global statistics identical on both ranks and equal to the single-rank run
    assert np.array_equal(s0[:nst], sa[:nst]) and np.array_equal(s1[:nst], sa[:nst])
    assert np.array_equal(np.concatenate([s0[nst:], s1[nst:]]), sa[nst:])  # per-env returns
    st0 = r0[:n_rows].reshape(STEPS, N_LOCAL, width)
    st1 = r1[:n_rows].reshape(STEPS, N_LOCAL, width)
    sta = a[:2 * n_rows].reshape(STEPS, 2 * N_LOCAL, width)
    assert np.array_equal(np.concatenate([st0, st1], 1), sta)
    z0 = r0[n_rows:n_rows + N_LOCAL * DIM]
    z1 = r1[n_rows:n_rows + N_LOCAL * DIM]
    za = a[2 * n_rows:2 * n_rows + 2 * N_LOCAL * DIM]
    assert np.array_equal(np.concatenate([z0, z1]), za)
