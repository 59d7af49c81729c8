"""GPU: graph capture of the step and the multi-GPU shard path, through the C ABI.

- A HIP graph holding K env-steps (captured with torch.cuda.graph) replayed 100 times must equal the
  same steps run eagerly, every step, and the oracle at the end -- with the compact tier's overflow
  fallback forced on (diagnostic contact cap), so the device-resident overflow list is emptied and
  refilled inside every replay.  K = 3 is odd on purpose: the round-1 host-side step parity baked
  into a captured odd-length sequence never re-zeroed its counter (the recorded replay hang).
- A Batch holding global envs [4096, 8192) (env_id_offset = 4096) must equal rows 4096..8191 of an
  8192-env unsharded Batch for 200 env-steps with auto-resets (per-env results are
  invariant to the GPU count).
- ShardedEnvs over RCCL (backend "nccl") at world size 1 -- scatter of actions, gather of the
  payload through the collective -- equals the plain Batch, for the 24-d and 13-d ids.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LO = np.array([0.04799994, -0.11650084, 0.0, 0.0])
HI = np.array([0.54799994, 0.38349916, 0.5, 1.0])


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _grasp_actions(rng, n):
    a = np.zeros((n, 4))
    a[:, 0] = 0.29799994 + rng.normal(size=n) * 0.01
    a[:, 1] = 0.13349916 + rng.normal(size=n) * 0.01
    a[:, 2] = rng.uniform(0.02, 0.12, size=n)
    a[:, 3] = rng.uniform(0.5, 1.0, size=n)
    return a


def _eq(torch, x, y, what):
    assert torch.equal(x, y), f"{what}: max diff {(x.double() - y.double()).abs().max().item()}"


@pytest.mark.parametrize("schedule", [0, 2])
def test_graph_capture_replay_bit_exact(schedule):
    """schedule 2 captures the substep work queue (its unit counters and epoch live on the device)"""
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n, K, R = 128, 3, 100
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=21, tier_con_cap=2,
                         max_episode_steps=40, schedule=schedule)
    ge = rt.Batch(mc, cfg, n)
    gg = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    dev = ge.obs.device
    static_a = torch.zeros((K, n, 4), dtype=torch.float64, device=dev)
    graph = torch.cuda.CUDAGraph()
    snaps = []
    with torch.cuda.graph(graph):
        for k in range(K):
            out = gg.step(static_a[k])
            snaps.append(tuple(x.clone() for x in out))  # the batch's buffers are rewritten every step
    rng = np.random.default_rng(4)
    n_done = 0
    for r in range(R):
        a = np.stack([_grasp_actions(rng, n) if (r % 2) else rng.uniform(LO, HI, size=(n, 4)) for _ in range(K)])
        at = torch.from_numpy(a).to(dev)
        static_a.copy_(at)
        graph.replay()
        for k in range(K):
            e_obs, e_rew, e_term, e_trunc, e_tobs = ge.step(at[k])
            o_obs, o_rew, o_term, o_trunc, o_tobs = ob.step(a[k])
            g_obs, g_rew, g_term, g_trunc, g_tobs = snaps[k]
            _eq(torch, g_obs, e_obs, f"obs replay {r} step {k}")
            _eq(torch, g_rew, e_rew, f"reward replay {r} step {k}")
            _eq(torch, g_term, e_term, f"terminated replay {r} step {k}")
            _eq(torch, g_trunc, e_trunc, f"truncated replay {r} step {k}")
            done = (e_term | e_trunc) > 0
            _eq(torch, g_tobs[done], e_tobs[done], f"terminal obs replay {r} step {k}")
            n_done += int(done.sum())
            np.testing.assert_array_equal(g_obs.cpu().numpy(), o_obs, err_msg=f"obs vs oracle replay {r} step {k}")
            np.testing.assert_array_equal(g_rew.cpu().numpy(), o_rew, err_msg=f"reward vs oracle replay {r}")
        for x, y, what in zip(gg.get_state(), ge.get_state(), ("qpos", "qvel", "warmstart")):
            _eq(torch, x, y, f"{what} after replay {r}")
    torch.cuda.synchronize()
    oqp, oqv, owa, onc = ob.get_state()
    qp, qv, wa = gg.get_state()
    np.testing.assert_array_equal(qp.cpu().numpy(), oqp)
    np.testing.assert_array_equal(qv.cpu().numpy(), oqv)
    np.testing.assert_array_equal(wa.cpu().numpy(), owa)
    np.testing.assert_array_equal(gg.get_info()["ncon"].cpu().numpy(), onc)
    ovf_g, ovf_e = gg.overflow_count(), ge.overflow_count()
    assert ovf_g == ovf_e and ovf_g > 0, (ovf_g, ovf_e)  # the fallback ran inside the replays
    assert n_done > 0
    gg.close()
    ge.close()


def test_shard_offset_matches_unsharded_rows():
    torch = _torch()
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n_full, off, steps = 8192, 4096, 200
    kw = dict(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=77, max_episode_steps=60)
    full = rt.Batch(mc, rt.make_config(**kw), n_full)
    shard = rt.Batch(mc, rt.make_config(env_id_offset=off, **kw), n_full - off)
    _eq(torch, shard.obs, full.obs[off:], "reset obs")
    dev = full.obs.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    lo = torch.tensor(LO, device=dev)
    hi = torch.tensor(HI, device=dev)
    n_done = 0
    for s in range(steps):
        a = lo + (hi - lo) * torch.rand((n_full, 4), dtype=torch.float64, device=dev, generator=gen)
        f = full.step(a)
        g = shard.step(a[off:])
        for x, y, what in zip(g[:4], f[:4], ("obs", "reward", "terminated", "truncated")):
            _eq(torch, x, y[off:], f"{what} step {s}")
        done = (g[2] | g[3]) > 0
        _eq(torch, g[4][done], f[4][off:][done], f"terminal obs step {s}")
        n_done += int(done.sum())
    for x, y, what in zip(shard.get_state(), full.get_state(), ("qpos", "qvel", "warmstart")):
        _eq(torch, x, y[off:], what)
    _eq(torch, shard.get_info()["ncon"], full.get_info()["ncon"][off:], "ncon")
    assert n_done > n_full - off  # every env truncates at least once (T = 60)
    full.close()
    shard.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("env_id", ["gymnasium_env/ur3e-v2", "gymnasium_env/ur3e-v0"])
def test_sharded_envs_rccl_self_gather(env_id):
    torch = _torch()
    import torch.distributed as dist
    from ur3e_amd import runtime as rt
    from ur3e_amd.envs.sharded import ShardedEnvs
    from ur3e_amd.envs.specs import spec
    sp = spec(env_id)
    md, mc = rt.load_model("main")
    n = 512
    cfg = rt.make_config(task=sp["task"], frame_skip=sp["frame_skip"], max_episode_steps=30, model=md, seed=9,
                         task_gains=sp["gains"])
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        local = rt.Batch(mc, cfg, n)
        plain = rt.Batch(mc, cfg, n)
        env = ShardedEnvs(local, n)
        assert env.obs_dim == sp["obs_dim"] and env.act_dim == 4
        _eq(torch, env.reset(), plain.reset(), "reset obs")
        rng = np.random.default_rng(2)
        n_done = 0
        for s in range(100):
            a = torch.from_numpy(rng.uniform(sp["low"], sp["high"], size=(n, 4))).cuda()
            r = env.step(a)
            p = plain.step(a)
            for x, y, what in zip(r[:2], p[:2], ("obs", "reward")):
                _eq(torch, x, y, f"{what} step {s}")
            _eq(torch, r[2], p[2] > 0, f"terminated step {s}")
            _eq(torch, r[3], p[3] > 0, f"truncated step {s}")
            done = (p[2] | p[3]) > 0
            _eq(torch, r[4][done], p[4][done], f"terminal obs step {s}")
            n_done += int(done.sum())
        assert n_done > 0
        local.close()
        plain.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,cap", [(777, 0), (4096, 0), (512, 3)])
def test_substep_queue_matches_env_step_launch(n, cap):
    """The substep work queue (w_env_step_q: (substep, env) units, state handed over through HBM
    between substeps; the default launch above the resident slot count, forced here by schedule 2)
    must
    equal the one-workgroup-per-env-step launch (schedule 1) bit for bit, every step, including
    envs that bail to the full-capacity tier in either substep (cap = diagnostic contact cap) and
    auto-resets; n = 777 is not a multiple of the 8 XCDs."""
    torch = _torch()
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    kw = dict(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=17, max_episode_steps=40, tier_con_cap=cap)
    gq = rt.Batch(mc, rt.make_config(schedule=2, **kw), n)
    ge = rt.Batch(mc, rt.make_config(schedule=1, **kw), n)
    _eq(torch, gq.obs, ge.obs, "reset obs")
    rng = np.random.default_rng(8)
    for s in range(60):
        a = _grasp_actions(rng, n) if s % 3 else rng.uniform(LO, HI, size=(n, 4))
        at = torch.from_numpy(a).cuda()
        q = gq.step(at)
        e = ge.step(at)
        for x, y, what in zip(q[:4], e[:4], ("obs", "reward", "terminated", "truncated")):
            _eq(torch, x, y, f"{what} step {s}")
        done = (e[2] | e[3]) > 0
        _eq(torch, q[4][done], e[4][done], f"terminal obs step {s}")
    for x, y, what in zip(gq.get_state(), ge.get_state(), ("qpos", "qvel", "warmstart")):
        _eq(torch, x, y, what)
    _eq(torch, gq.get_info()["ncon"], ge.get_info()["ncon"], "ncon")
    oq, oe = gq.overflow_count(), ge.overflow_count()
    if cap:
        assert oq > 0 and oe > 0
    gq.close()
    ge.close()


def test_graph_capture_grasp_routing():
    """The tier routing inside a captured step: the scripted pick (C3 semantics) in its grasp rows,
    where envs hold 12-20 contacts, so each step routes them to the grasp tier on the library's
    internal stream (fork/join events inside the graph) while the compact tier skips them.  A
    3-step graph replayed 60 times over rows 1850..2030 must equal the same rows stepped eagerly and
    the oracle, with routed env-steps counted inside the replays."""
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd.controller.move_l_mug import MoveLMug
    n, K, R, r0 = 32, 3, 60, 1850
    de = MoveLMug(n, reset_mode="low", seed=5)
    dg = MoveLMug(n, reset_mode="low", seed=5)
    ob = po.OracleBatch(de.batch.model_c, po.config_from(de.batch.cfg), n)
    for t in range(r0):
        row = de.traj.row(t)
        de.batch.step(row)
        dg.batch.step(row)
        ob.step(row.cpu().numpy())
    dev = de.batch.obs.device
    static_a = torch.zeros((K, n, 7), dtype=torch.float64, device=dev)
    graph = torch.cuda.CUDAGraph()
    snaps = []
    with torch.cuda.graph(graph):
        for k in range(K):
            out = dg.batch.step(static_a[k])
            snaps.append(out[0].clone())
    routed0 = dg.batch.tier_counts()[2] + dg.batch.mid_count()
    t = r0
    for r in range(R):
        rows = torch.stack([de.traj.row(t + k) for k in range(K)])
        static_a.copy_(rows)
        graph.replay()
        for k in range(K):
            e_obs = de.batch.step(rows[k])[0]
            o_obs = ob.step(rows[k].cpu().numpy())[0]
            _eq(torch, snaps[k], e_obs, f"obs replay {r} step {k}")
            np.testing.assert_array_equal(snaps[k].cpu().numpy(), o_obs, err_msg=f"obs vs oracle replay {r} step {k}")
        t += K
        for x, y, what in zip(dg.batch.get_state(), de.batch.get_state(), ("qpos", "qvel", "warmstart")):
            _eq(torch, x, y, f"{what} after replay {r}")
    torch.cuda.synchronize()
    oqp, oqv, owa, onc = ob.get_state()
    qp, qv, wa = dg.batch.get_state()
    np.testing.assert_array_equal(qp.cpu().numpy(), oqp)
    np.testing.assert_array_equal(qv.cpu().numpy(), oqv)
    np.testing.assert_array_equal(dg.batch.get_info()["ncon"].cpu().numpy(), onc)
    # envs were routed past the compact tier (to the mid or the grasp tier) inside the replays
    assert dg.batch.tier_counts()[2] + dg.batch.mid_count() > routed0
    assert int(onc.max()) > 10  # the grasp exceeded the compact tier's contact capacity
    de.close()
    dg.close()
