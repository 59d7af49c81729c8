"""Multi-rank sharding (world_size 2, gloo, CPU): per-env results must equal a
single-rank run over the same global env ids (reset noise is keyed by global
id), with actions scattered from and results gathered to rank 0."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_local, steps, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from tests.helpers import OracleStepper
    from ur3e_amd.envs.sharded import ShardedEnvs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = OracleStepper(n_local, seed=5, env_id_offset=rank * n_local, max_episode_steps=4)
    env = ShardedEnvs(local, n_local)
    obs0 = env.reset()
    rng = np.random.default_rng(1)
    res = []
    for _ in range(steps):
        a = torch.from_numpy(rng.uniform([0.05, -0.1, 0, 0], [0.5, 0.38, 0.5, 1], size=(n_local * world, 4)))
        r = env.step(a if rank == 0 else None)
        if rank == 0:
            res.append(torch.cat([r[0], r[1][:, None], r[2][:, None].double(), r[3][:, None].double()], 1).numpy())
    if rank == 0:
        np.save(out_path, np.stack(res, 0))
        np.save(out_path + ".obs0.npy", obs0.numpy())
    dist.destroy_process_group()


def test_sharding_invariance(tmp_path):
    import torch
    from tests.helpers import OracleStepper
    n_local, world, steps = 3, 2, 6
    out = str(tmp_path / "g.npy")
    mp.spawn(_worker, args=(world, _free_port(), n_local, steps, out), nprocs=world, join=True)
    got = np.load(out)
    obs0 = np.load(out + ".obs0.npy")
    # single-rank reference over the same 6 global envs
    ref = OracleStepper(n_local * world, seed=5, max_episode_steps=4)
    np.testing.assert_array_equal(obs0, ref.reset().numpy())
    rng = np.random.default_rng(1)
    for s in range(steps):
        a = torch.from_numpy(rng.uniform([0.05, -0.1, 0, 0], [0.5, 0.38, 0.5, 1], size=(n_local * world, 4)))
        o, r, te, tr, _ = ref.step(a)
        exp = torch.cat([o, r[:, None], te[:, None].double(), tr[:, None].double()], 1).numpy()
        np.testing.assert_array_equal(got[s], exp)
