"""GPU: the substep work queue (w_env_step_q) -- forward progress and its trace build, through the C ABI.

- Two handles on two streams step 4,096 envs each concurrently (the two queue launches share the
  GPU's workgroup slots, so static first units can belong to workgroups that are not resident): the
  results equal the same handles stepped one after the other, and no unit gives up.
- The same with most workgroup slots held by a third stream (ur3e_debug_hold_slots: 64 KB-LDS
  workgroups that stay resident for a few ms, launched and waited for until they all run), so that the
  queue launches find only one slot per CU: workgroups whose static units are not resident yet, and the
  consumers claim them.  Claims must happen, nothing gives up, and results equal the sequential runs.
- Owners that leave their static units to the consumers (diagnostic): every static unit is claimed
  and run by its substep-1 unit, bit-exact against the oracle.
- A diagnostic spin limit of a few polls forces the give-up path: the envs go to the fallback tiers,
  which recompute the env-step -- bit-exact against the oracle, and the give-ups are counted.
- The queue-trace build (unit stamps stored by lane 0 inside the queue kernel's loop) runs at 4,096
  envs bit-exact against the product library and stamps every unit.
- Split last substeps (ur3e_batch_set_queue_split): with none, half and all of each queue's envs running
  their last substep as two half units (the working set handed between workgroups through HBM), the
  results are bit-exact against the oracle, auto-resets inside the resumed halves included; the trace
  build stamps the second halves too.
"""
import ctypes
import os

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


def _eq(torch, x, y, what):
    assert torch.equal(x, y), f"{what}: max diff {(x.double() - y.double()).abs().max().item()}"


def _snap(b):
    qp, qv, wa = b.get_state()
    return [b.obs.clone(), b.reward.clone(), b.terminated.clone(), b.truncated.clone(), qp, qv, wa]


def _cmp(torch, a, b, what):
    for k, (x, y) in enumerate(zip(a, b)):
        _eq(torch, x, y, f"{what} field {k}")


def test_two_handles_two_streams_concurrent():
    torch = _torch()
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n, steps = 4096, 50
    cfgs = [rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=s, max_episode_steps=30)
            for s in (3, 4)]
    gen = torch.Generator(device="cuda").manual_seed(7)
    lo = torch.tensor(LO, device="cuda")
    hi = torch.tensor(HI, device="cuda")
    acts = [[lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda", generator=gen)
             for _ in range(steps)] for _ in range(2)]
    # one after the other (default stream)
    seq = []
    for h in range(2):
        b = rt.Batch(mc, cfgs[h], n)
        assert b.kernel_info()["kernel"].startswith("w_env_step_q")
        for t in range(steps):
            b.step(acts[h][t])
        torch.cuda.synchronize()
        seq.append(_snap(b))
        b.close()
    # concurrently: handle h enqueues on its own stream, the two streams interleaved step by step
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bs = [rt.Batch(mc, cfgs[h], n) for h in range(2)]
    torch.cuda.synchronize()
    for t in range(steps):
        for h in range(2):
            with torch.cuda.stream(streams[h]):
                bs[h].step(acts[h][t])
    torch.cuda.synchronize()
    for h in range(2):
        _cmp(torch, _snap(bs[h]), seq[h], f"handle {h}")
        giveups, claimed = bs[h].queue_stats()
        assert giveups == 0, f"handle {h}: {giveups} queue units gave up"
        print(f"handle {h}: static units claimed by consumers: {claimed}")
        bs[h].close()


def test_queue_with_slots_held_claims_static_units():
    torch = _torch()
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n, steps = 4096, 12
    cfgs = [rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=s, max_episode_steps=30)
            for s in (13, 14)]
    gen = torch.Generator(device="cuda").manual_seed(17)
    lo = torch.tensor(LO, device="cuda")
    hi = torch.tensor(HI, device="cuda")
    acts = [[lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda", generator=gen)
             for _ in range(steps)] for _ in range(2)]
    seq = []
    for h in range(2):
        b = rt.Batch(mc, cfgs[h], n)
        for t in range(steps):
            b.step(acts[h][t])
        torch.cuda.synchronize()
        seq.append(_snap(b))
        b.close()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    holder = torch.cuda.Stream()
    bs = [rt.Batch(mc, cfgs[h], n) for h in range(2)]
    torch.cuda.synchronize()
    props = torch.cuda.get_device_properties(0)
    n_hold = 2 * props.multi_processor_count  # two 64 KB workgroups per CU
    started = []
    for t in range(steps):
        # slots held before every other step's launches (the hold outlasts a launch: 3 ms)
        if t % 2 == 0:
            started.append(rt.hold_slots(n_hold, 3000, stream=holder))
        for h in range(2):
            with torch.cuda.stream(streams[h]):
                bs[h].step(acts[h][t])
    torch.cuda.synchronize()
    print(f"hold workgroups started before the launches: {started} of {n_hold}")
    assert max(started) >= n_hold // 2
    claimed_total = 0
    for h in range(2):
        _cmp(torch, _snap(bs[h]), seq[h], f"handle {h}")
        giveups, claimed = bs[h].queue_stats()
        assert giveups == 0, f"handle {h}: {giveups} queue units gave up"
        print(f"handle {h}: static units claimed by consumers: {claimed}")
        claimed_total += claimed
        bs[h].close()
    assert claimed_total > 0, "the held slots never left a static unit to its consumer"


@pytest.mark.parametrize("mode", ["leave_static", "spin_limit"])
def test_queue_claim_and_giveup_paths_bit_exact(mode):
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n, steps = 512, 12
    # schedule 2: the queue at any env count (512 envs -> 1,024 workgroups: 64 static units per queue)
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=9, max_episode_steps=8, schedule=2)
    g = rt.Batch(mc, cfg, n)
    assert g.kernel_info()["kernel"].startswith("w_env_step_q")
    if mode == "leave_static":
        g.set_queue_debug(leave_static_units=True)
    else:
        g.set_queue_debug(spin_limit=2)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(5)
    for t in range(steps):
        a = rng.uniform(LO, HI, size=(n, 4))
        o = ob.step(a)
        g.step(torch.from_numpy(a))
        torch.cuda.synchronize()
        assert np.array_equal(g.obs.cpu().numpy(), o[0]), f"obs step {t}"
        assert np.array_equal(g.reward.cpu().numpy(), o[1]), f"reward step {t}"
        assert np.array_equal(g.terminated.cpu().numpy(), o[2]) and np.array_equal(g.truncated.cpu().numpy(), o[3])
    qp, qv, wa = g.get_state()
    oqp, oqv, owa, _ = ob.get_state()
    assert np.array_equal(qp.cpu().numpy(), oqp) and np.array_equal(qv.cpu().numpy(), oqv)
    assert np.array_equal(wa.cpu().numpy(), owa)
    giveups, claimed = g.queue_stats()
    if mode == "leave_static":
        assert giveups == 0
        # every static unit of every step (64 per queue), less those of envs routed to the grasp tier
        assert 0.9 * 64 * 8 * steps <= claimed <= 64 * 8 * steps, claimed
    else:
        assert giveups > 0, "the small spin limit never gave up"
        assert g.tier_counts()[0] >= giveups  # each give-up went to the fallback tiers
    g.close()


def test_trace_build_queue_4096_bit_exact():
    torch = _torch()
    from ur3e_amd import _build
    from ur3e_amd import runtime as rt
    if not os.path.exists(_build.TRACE_LIB):
        pytest.fail(f"trace build missing: {_build.TRACE_LIB} (built by __graft_entry__.build())")
    md, mc = rt.load_model("main")
    n, steps = 4096, 6
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=13)
    gp = rt.Batch(mc, cfg, n)
    gt = rt.Batch(mc, cfg, n, lib=_build.TRACE_LIB)
    assert gt.kernel_info()["kernel"].startswith("w_env_step_q")
    gp.set_queue_split(0)
    gt.set_queue_split(100)  # every env's last substep in two halves: rows 2n.. hold the second halves
    gen = torch.Generator(device="cuda").manual_seed(3)
    lo = torch.tensor(LO, device="cuda")
    hi = torch.tensor(HI, device="cuda")
    nrow = 3 * n
    tr = np.zeros((nrow, 4), dtype=np.uint64)
    for t in range(steps):
        a = lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda", generator=gen)
        gp.step(a)
        gt.step(a)
        torch.cuda.synchronize()
        _cmp(torch, _snap(gt), _snap(gp), f"step {t}")
    assert gt.L.ur3e_debug_wave_trace(tr.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), nrow) == 0
    # the units of the last launch were pulled, acquired and finished in that order (envs routed to
    # the grasp tier keep older stamps, or none: a few percent in the first steps after the reset, while
    # the dropped mugs land with more contacts than the compact tier takes)
    pulled, acquired, finished = (tr[:, k].astype(np.int64) for k in range(3))
    done = (pulled > 0) & (acquired > 0) & (finished > 0)
    print("units stamped:", done.mean(), "tier counts:", gt.tier_counts())
    assert done.mean() > 0.9, done.mean()
    assert (finished[done] >= acquired[done]).all() and (acquired[done] >= pulled[done]).all()
    # a second half acquires its env after its first half did (the hand-off flag; the first half's own
    # "finished" stamp is taken after its release, and after pulling its next unit, so it may come later)
    both = done[n:2 * n] & done[2 * n:]
    assert both.mean() > 0.9, both.mean()
    assert (acquired[2 * n:][both] >= acquired[n:2 * n][both]).all()
    gp.close()
    gt.close()


def test_queue_split_units_bit_exact():
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n, steps = 4096, 12
    # short episodes: the auto-reset runs inside resumed second halves
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=23, max_episode_steps=7)
    gs = []
    for pct in (0, 50, 100):
        g = rt.Batch(mc, cfg, n)
        assert g.kernel_info()["kernel"].startswith("w_env_step_q")
        g.set_queue_split(pct)
        gs.append(g)
    with pytest.raises(RuntimeError):
        gs[0].set_queue_split(101)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(29)
    for t in range(steps):
        a = rng.uniform(LO, HI, size=(n, 4))
        o = ob.step(a)
        at = torch.from_numpy(a)
        for g in gs:
            g.step(at)
        torch.cuda.synchronize()
        for pct, g in zip((0, 50, 100), gs):
            assert np.array_equal(g.obs.cpu().numpy(), o[0]), f"split {pct}: obs step {t}"
            assert np.array_equal(g.reward.cpu().numpy(), o[1]), f"split {pct}: reward step {t}"
            assert np.array_equal(g.terminated.cpu().numpy(), o[2]), f"split {pct}: terminated step {t}"
            assert np.array_equal(g.truncated.cpu().numpy(), o[3]), f"split {pct}: truncated step {t}"
    oqp, oqv, owa, _ = ob.get_state()
    for pct, g in zip((0, 50, 100), gs):
        qp, qv, wa = g.get_state()
        assert np.array_equal(qp.cpu().numpy(), oqp) and np.array_equal(qv.cpu().numpy(), oqv), f"split {pct}"
        assert np.array_equal(wa.cpu().numpy(), owa), f"split {pct}"
        assert g.queue_stats()[0] == 0
        g.close()
