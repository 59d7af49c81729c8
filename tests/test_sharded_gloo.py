"""Multi-rank sharding (world_size 2, gloo, CPU): per-env results must equal a
single-rank run over the same global env ids (reset noise is keyed by global
id), with actions scattered from and results gathered to rank 0.  Covered for
every observation / action width the registered ids have: ur3e-v2 (24 / 4),
ur3e-v0 (13 / 4) and imitation_direct-v0 (13 / 7 raw controls)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _actions(rng, env_id, n):
    from ur3e_amd.envs.specs import spec
    s = spec(env_id)
    return rng.uniform(s["low"], s["high"], size=(n, len(s["low"])))


def _worker(rank, world, port, n_local, steps, env_id, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from tests.helpers import OracleStepper
    from ur3e_amd.envs.sharded import ShardedEnvs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = OracleStepper(n_local, seed=5, env_id_offset=rank * n_local, max_episode_steps=4, env_id=env_id)
    env = ShardedEnvs(local, n_local)
    assert env.obs_dim == local.obs_dim and env.act_dim == local.act_dim
    obs0 = env.reset()
    rng = np.random.default_rng(1)
    res = []
    for _ in range(steps):
        a = torch.from_numpy(_actions(rng, env_id, n_local * world))
        r = env.step(a if rank == 0 else None)
        if rank == 0:
            res.append(torch.cat([r[0], r[1][:, None], r[2][:, None].double(), r[3][:, None].double(), r[4]],
                                 1).numpy().copy())
    if rank == 0:
        np.save(out_path, np.stack(res, 0))
        np.save(out_path + ".obs0.npy", obs0.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("env_id", ["gymnasium_env/ur3e-v2", "gymnasium_env/ur3e-v0",
                                    "gymnasium_env/imitation_direct-v0"])
def test_sharding_invariance(tmp_path, env_id):
    import torch
    from tests.helpers import OracleStepper
    n_local, world, steps = 3, 2, 6
    out = str(tmp_path / "g.npy")
    mp.spawn(_worker, args=(world, _free_port(), n_local, steps, env_id, out), nprocs=world, join=True)
    got = np.load(out)
    obs0 = np.load(out + ".obs0.npy")
    # single-rank reference over the same 6 global envs
    ref = OracleStepper(n_local * world, seed=5, max_episode_steps=4, env_id=env_id)
    np.testing.assert_array_equal(obs0, ref.reset().numpy())
    rng = np.random.default_rng(1)
    n_done = 0
    for s in range(steps):
        a = torch.from_numpy(_actions(rng, env_id, n_local * world))
        o, r, te, tr, to = ref.step(a)
        done = (te | tr).numpy() > 0
        n_done += int(done.sum())
        exp = torch.cat([o, r[:, None], te[:, None].double(), tr[:, None].double()], 1).numpy()
        od = o.shape[1]
        np.testing.assert_array_equal(got[s][:, :od + 3], exp)
        np.testing.assert_array_equal(got[s][done, od + 3:], to.numpy()[done])
    assert n_done > 0  # the horizon of 4 forces auto-resets inside the window
