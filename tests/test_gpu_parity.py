"""GPU parity: the MI355X library (through its C ABI) vs the CPU oracle, same
seeded inputs.  The bar is bit-exactness: both sides run the same FP64
operation order with contraction off and deterministic transcendentals, so
qpos/qvel/obs/reward and the integer contact counts must match exactly.
(The north_star tolerance, |dqpos| <= 1e-5 after 1000 steps, is checked too,
but exact equality is what these tests require.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _oracle_cfg(po, c):
    return po.config_from(c)


def _run_pair(model_name, task, n, steps, action_fn, frame_skip=2, seed=7, epb=0, check_every=1, tier_con_cap=0,
              task_gains=None, max_episode_steps=2500, np_chunk_lanes=0):
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model(model_name)
    cfg = rt.make_config(task=task, frame_skip=frame_skip, model=md, seed=seed, envs_per_block=epb,
                         tier_con_cap=tier_con_cap, task_gains=task_gains, max_episode_steps=max_episode_steps,
                         np_chunk_lanes=np_chunk_lanes,
                         reset_noise=(model_name == "main"),
                         reset_key=md["id_key_down"] if md["id_key_down"] >= 0 else -1)
    gb = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, _oracle_cfg(po, cfg), n)
    gobs = gb.obs.cpu().numpy()
    gym = task in (rt.TASK_GYM_V2, rt.TASK_GYM_V0, rt.TASK_IMIT_INDIRECT, rt.TASK_IMIT_DIRECT)
    assert gb.obs_dim == ob.od
    if gym:
        np.testing.assert_array_equal(gobs, ob.obs)
    rng = np.random.default_rng(seed)
    max_dq = 0.0
    max_touch = [0.0]
    n_done = 0
    for s in range(steps):
        a = action_fn(rng, n, md)
        o_obs, o_rew, o_term, o_trunc, o_tobs = ob.step(a)
        g_obs, g_rew, g_term, g_trunc, g_tobs = gb.step(torch.from_numpy(a))
        if s % check_every == 0 or s == steps - 1:
            torch.cuda.synchronize()
            n_done += int(((o_term > 0) | (o_trunc > 0)).sum())
            qp, qv, wa = gb.get_state()
            oqp, oqv, owa, onc = ob.get_state()
            bad = np.flatnonzero((qp.cpu().numpy() != oqp).any(axis=1))
            assert bad.size == 0, f"qpos step {s}: envs {bad[:10]} ncon gpu {gb.get_info()['ncon'].cpu().numpy()[bad[:10]]} oracle {onc[bad[:10]]}"
            if gym:
                np.testing.assert_array_equal(g_tobs.cpu().numpy()[o_term | o_trunc > 0],
                                              o_tobs[o_term | o_trunc > 0], err_msg=f"terminal obs step {s}")
                np.testing.assert_array_equal(g_rew.cpu().numpy(), o_rew, err_msg=f"reward step {s}")
                np.testing.assert_array_equal(g_term.cpu().numpy(), o_term, err_msg=f"terminated step {s}")
                np.testing.assert_array_equal(g_trunc.cpu().numpy(), o_trunc, err_msg=f"truncated step {s}")
                np.testing.assert_array_equal(g_obs.cpu().numpy(), o_obs, err_msg=f"obs step {s}")
            max_dq = max(max_dq, float(np.abs(qp.cpu().numpy() - oqp).max()))
            np.testing.assert_array_equal(qp.cpu().numpy(), oqp, err_msg=f"qpos step {s}")
            np.testing.assert_array_equal(qv.cpu().numpy(), oqv, err_msg=f"qvel step {s}")
            np.testing.assert_array_equal(wa.cpu().numpy(), owa, err_msg=f"warmstart step {s}")
            info = gb.get_info()
            np.testing.assert_array_equal(info["ncon"].cpu().numpy(), onc, err_msg=f"ncon step {s}")
            if mc.ntouch > 0:
                gt = gb.get_touch().cpu().numpy()
                ot = np.stack([ob.diag(i)["touch"][:mc.ntouch] for i in range(n)])
                np.testing.assert_array_equal(gt, ot, err_msg=f"touch step {s}")
                max_touch[0] = max(max_touch[0], float(ot.max()))
    assert max_dq <= 1e-5
    gb.ovf = gb.overflow_count()
    gb.tiers = gb.tier_counts()
    gb.n_done = n_done
    gb.max_touch = max_touch[0]
    gb.close()
    return gb


def _gym_actions(rng, n, md):
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    return rng.uniform(lo, hi, size=(n, 4))


# kernel layouts: 0 = two-tier (compact 64-lane tier + full-capacity fallback, default),
# -128 / -64 = full-capacity tier only with 128 / 64 lanes per env, 16 = one env per lane (v1)
@pytest.mark.parametrize("epb", [0, -128, -64, 16])
def test_gym_v2_random_actions_short(epb):
    _run_pair("main", 0, 64, 60, _gym_actions, epb=epb)


@pytest.mark.parametrize("n", [1, 13, 24])
def test_gym_v2_env_counts(n):
    """Env counts that are not / are multiples of the 8 XCDs: the step kernel's XCD-aware env order
    is the identity for 1 and 13 envs and a real permutation for 24 (workgroup b -> env
    (b % 8) * 3 + b / 8); every env must still match the oracle bit for bit."""
    _run_pair("main", 0, n, 40, _gym_actions, seed=5)


def _grasp_actions(rng, n, md):
    # actions concentrated around the mug with the gripper closing: exercises pad-box contacts
    a = np.zeros((n, 4))
    a[:, 0] = 0.29799994 + rng.normal(size=n) * 0.01
    a[:, 1] = 0.13349916 + rng.normal(size=n) * 0.01
    a[:, 2] = rng.uniform(0.02, 0.12, size=n)
    a[:, 3] = rng.uniform(0.5, 1.0, size=n)
    return a


def test_gym_v2_grasp_region():
    _run_pair("main", 0, 64, 150, _grasp_actions, seed=3)


@pytest.mark.parametrize("lanes", [1, 3])
def test_narrowphase_chunks(lanes):
    """The compact tier's narrowphase runs survivor pairs in chunks of up to 8 lanes (clip
    polygons and the contact stage live in LDS per chunk). With the diagnostic chunk width 1 or 3
    every env with contacts goes through several chunks; contacts must still come out in
    candidate order, bit-exact against the oracle."""
    _run_pair("main", 0, 64, 100, _grasp_actions, seed=3, np_chunk_lanes=lanes)


@pytest.mark.parametrize("cap", [2, 3, -2])
def test_two_tier_fallback(cap):
    """Compact-tier overflow mid-step (the diagnostic cap makes envs with more than `cap` contacts
    overflow in either substep or in an auto-reset) hands the env to the grasp tier (cap > 0) or,
    when the grasp tier is capped too (cap < 0), on to the full-capacity tier; each recomputes the
    step from the untouched state: results stay bit-exact, the fallback is taken, including
    mid-step bails after a substep already ran."""
    gb = _run_pair("main", 0, 64, 80, _grasp_actions, seed=11, tier_con_cap=cap)
    assert gb.ovf > 0 and gb.tiers[0] == gb.ovf
    if cap > 0:
        assert gb.tiers[1] == 0  # the grasp tier held every env the compact tier handed on
    else:
        assert gb.tiers[1] > 0  # ... and with it capped the envs reached the full-capacity tier


def test_move_j_2f85():
    def act(rng, n, md):
        q0 = np.array(md["key_qpos"][md["id_key_down"]][:6])
        a = np.zeros((n, 7))
        a[:, :6] = q0 + rng.uniform(-0.5, 0.5, size=(n, 6))
        a[:, 6] = rng.uniform(0, 1, size=n)
        return a
    _run_pair("ur3e_2f85", 2, 64, 100, act)


def _traj_follower(rows, n, noise, seed=3):
    """action_fn replaying trajectory rows (one row per env-step, row index = step), with a fixed
    per-env offset on the position columns so the envs differ"""
    off = np.random.default_rng(seed).normal(size=(n, 3)) * noise
    state = {"t": 0}

    def act(rng, n_, md):
        r = rows[min(state["t"], len(rows) - 1)]
        state["t"] += 1
        a = np.tile(r, (n_, 1))
        a[:, :3] += off
        return a
    return act


def test_move_l_2f85_traj_l():
    """move_l.main (controller/move_l.py:88-140) on ur3e_2f85: build_traj_l rows (seed 49 cubic path)
    through the move_l controller (pinv joint deltas + two pd_joint_ctrl calls), 1 physics step per
    row, bit-exact vs the oracle.  The trajectory starts at the tcp pose of the reset state."""
    from ur3e_amd import runtime as rt
    from ur3e_amd.controller import build_traj as bt
    _torch()
    md, mc = rt.load_model("ur3e_2f85")
    probe = rt.Batch(mc, rt.make_config(task=rt.TASK_MOVE_L, model=md, reset_noise=None), 1)
    c = probe.get_carry().cpu().numpy()[0]
    probe.close()
    start = np.concatenate([c[0:3], [-1.209, -1.209, 1.209], [0.0]])
    rows = bt.build_traj_l(start, 1)  # one row per env-step (hold 1 keeps the 500-row path short)
    _run_pair("ur3e_2f85", rt.TASK_MOVE_L, 32, 300, _traj_follower(rows, 32, 0.01), check_every=5)


def test_move_j_raw_traj_j():
    """Config 1 (BASELINE.json configs[0]): ur3e_raw (arm only, dt 1e-4, qpos0 = 0), move_j PD with
    config_j.yml gains along build_traj_j(0, hold) rows; grip column dropped (nu = 6)."""
    from ur3e_amd.controller import build_traj as bt
    rows = bt.build_traj_j(np.zeros(7), 2)
    _run_pair("ur3e_raw", 2, 16, 400, _traj_follower(rows, 16, 0.0), check_every=10)


def test_ctrl_raw():
    def act(rng, n, md):
        return rng.uniform(-20, 20, size=(n, 6))
    _run_pair("ur3e_raw", 3, 32, 100, act, frame_skip=1)


def _v0_actions(rng, n, md):
    # ur3e_env.py:61-66 action Box ([x, y, z] around the mug + gripper)
    lo = np.array([0.28799994, 0.13349916, 0.005, 0.0])
    hi = np.array([0.35799994, 0.35349916, 0.165, 1.0])
    return rng.uniform(lo, hi, size=(n, 4))


def test_gym_v0_random_actions():
    """ur3e-v0 (task 4): 13-d obs, reward with self/table-collision terms, termination, truncation
    before the increment (T=40 here so auto-reset with the 13-d terminal observation runs)."""
    from ur3e_amd import runtime as rt
    gb = _run_pair("main", rt.TASK_GYM_V0, 64, 90, _v0_actions, task_gains=rt.GAINS_V0,
                   max_episode_steps=40, seed=5)
    assert gb.n_done > 0


def test_imitation_indirect():
    """imitation-indirect (task 5): v2 action Box through pid_task_ctrl, 24-d obs, reward -1."""
    from ur3e_amd import runtime as rt
    gb = _run_pair("main", rt.TASK_IMIT_INDIRECT, 64, 60, _gym_actions, frame_skip=1, max_episode_steps=25,
                   seed=9)
    assert gb.n_done > 0


def test_imitation_direct():
    """imitation-direct (task 6): raw ctrl inside actuator ctrlrange, 13-d obs, reward -1."""
    from ur3e_amd import runtime as rt

    def act(rng, n, md):
        cr = np.array(md["act_ctrlrange"])
        return rng.uniform(cr[:, 0], cr[:, 1], size=(n, cr.shape[0]))
    gb = _run_pair("main", rt.TASK_IMIT_DIRECT, 64, 60, act, max_episode_steps=25, seed=13)
    assert gb.n_done > 0


@pytest.mark.slow
def test_gym_v2_1000_steps():
    """north_star: qpos within 1e-5 after 1000 steps (here: bit-exact)."""
    _run_pair("main", 0, 128, 1000, _gym_actions, check_every=100)


def test_move_l_mug_scripted_pick():
    """C3 semantics (controller/move_l_mug.py): closed-loop pid_task_ctrl along per-env
    build_traj_l_pick_place rows, one mj_step per row, through the pick and most of the lift
    segment; GPU vs oracle bit-exact on state, contacts, touch sensors and the task-space obs,
    and the scripted grasp really happens: both pads on the mug (obs[23] robust grasp) and the
    mug lifted off the table."""
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    from ur3e_amd.controller.move_l_mug import MoveLMug, task_space_state
    n = 16
    drv = MoveLMug(n, reset_mode="low", seed=5)
    gb = drv.batch
    ob = po.OracleBatch(gb.model_c, _oracle_cfg(po, gb.cfg), n)
    np.testing.assert_array_equal(gb.obs.cpu().numpy(), ob.obs)
    max_touch = 0.0
    grasped = np.zeros(n, dtype=bool)
    z0 = gb.obs[:, 5].cpu().numpy().copy()
    steps = 3000
    for s in range(steps):
        row = drv.step()
        o_obs = ob.step(row.cpu().numpy())[0]
        if s % 250 == 0 or s == steps - 1:
            torch.cuda.synchronize()
            qp, qv, wa = gb.get_state()
            oqp, oqv, owa, onc = ob.get_state()
            np.testing.assert_array_equal(qp.cpu().numpy(), oqp, err_msg=f"qpos row {s}")
            np.testing.assert_array_equal(qv.cpu().numpy(), oqv, err_msg=f"qvel row {s}")
            np.testing.assert_array_equal(gb.get_info()["ncon"].cpu().numpy(), onc, err_msg=f"ncon row {s}")
            np.testing.assert_array_equal(gb.obs.cpu().numpy(), o_obs, err_msg=f"obs row {s}")
            gt = gb.get_touch().cpu().numpy()
            ot = np.stack([ob.diag(i)["touch"][:2] for i in range(n)])
            np.testing.assert_array_equal(gt, ot, err_msg=f"touch row {s}")
            max_touch = max(max_touch, float(gt.max()))
            grasped |= o_obs[:, 23] == 1.0
    assert grasped.sum() >= n // 4
    assert (gb.obs[:, 5].cpu().numpy() - z0).max() > 0.01
    # the firm grasp exceeds the compact tier (12-20 contacts): those env-steps ran in the grasp tier,
    # handed on by the compact tier or routed there by the previous step's contact count
    tc = gb.tier_counts()
    assert tc[0] + tc[2] > 0 and tc[2] > 0, tc
    st = task_space_state(gb)
    assert st.shape == (n, 7)
    drv.close()


@pytest.mark.parametrize("mode", ["indirect", "direct"])
def test_collect_demos_batched(mode):
    """collect_demos.py:86-189 batched: augmented-trajectory rows through pid_task_ctrl + one mj_step;
    recorded obs (get_obs) and actions ([x, y, z, u_grip] or the 7 ctrl) are bit-exact vs the oracle
    stepping the same rows, with down-sampling."""
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd.controller.collect_demos import DemoCollector
    n, steps, ds = 16, 700, 3
    col = DemoCollector(n, action_mode=mode, noise_mag="low", down_sample=ds, seed=2)
    gb = col.batch
    ob = po.OracleBatch(gb.model_c, _oracle_cfg(po, gb.cfg), n)
    np.testing.assert_array_equal(col.obs0.cpu().numpy(), ob.obs)
    rows = col.traj.traj[:steps].cpu().numpy()
    obs, acts = col.run(steps)
    obs, acts = obs.cpu().numpy(), acts.cpu().numpy()
    assert obs.shape == ((steps + ds - 1) // ds + 1, n, 24)
    j = 0
    for t in range(steps):
        o_obs = ob.step(rows[t])[0]
        if t % ds == 0:
            ctrl = np.stack([ob.diag(i)["ctrl"][:gb.nu] for i in range(n)])
            if mode == "indirect":
                exp = np.concatenate([rows[t][:, :3], ctrl[:, -1:]], axis=1)
            else:
                exp = ctrl
            np.testing.assert_array_equal(acts[j], exp, err_msg=f"acts row {t}")
            np.testing.assert_array_equal(obs[j + 1], o_obs, err_msg=f"obs row {t}")
            j += 1
    trajs = col.trajectories(torch.from_numpy(obs), torch.from_numpy(acts))
    assert len(trajs) == n and trajs[0].obs.shape[0] == trajs[0].acts.shape[0] + 1
    col.close()


@pytest.mark.parametrize("norm_reward,n", [(False, 1000), (True, 1000), (True, 20000)])
def test_vecnormalize_gpu_matches_sb3(norm_reward, n):
    """On-device VecNormalize (train_rl.py:57) vs the numpy restatement of SB3 2.7.0 on the same raw
    step outputs: running obs/return statistics, normalised f32 obs, rewards and terminal obs are
    bit-identical (numpy's axis-0 sequential and 1-D pairwise reduction orders)."""
    torch = _torch()
    from oracle.vecnorm_ref import VecNormalizeRef
    from ur3e_amd.envs.vec_env import UR3eVecEnv
    from ur3e_amd.envs.vec_normalize import VecNormalize
    # n = 1000 is not a multiple of 8 or 128: every branch of the pairwise sum; n = 20000 spans three
    # of numpy's 8192-element reduction buffers (the returns' sums are blocked like numpy's)
    venv = UR3eVecEnv(num_envs=n, seed=4, max_episode_steps=7)
    vn = VecNormalize(venv, norm_reward=norm_reward, clip_obs=10.0)
    ref = VecNormalizeRef(n, 24, norm_reward=norm_reward, clip_obs=10.0)
    o = vn.reset()
    np.testing.assert_array_equal(o, ref.reset(vn.get_original_obs()))
    rng = np.random.default_rng(0)
    saw_done = False
    for s in range(20):
        a = rng.uniform(venv.action_space.low, venv.action_space.high, size=(n, 4))
        obs, rew, dones, infos = vn.step(a)
        raw_obs, raw_rew = vn.get_original_obs(), vn.get_original_reward()
        raw_tobs = vn._last[2].cpu().numpy()
        r_obs, r_rew, r_tobs = ref.step(raw_obs, raw_rew, dones, raw_tobs)
        np.testing.assert_array_equal(vn.obs_rms.mean, ref.obs_rms.mean, err_msg=f"obs mean {s}")
        np.testing.assert_array_equal(vn.obs_rms.var, ref.obs_rms.var, err_msg=f"obs var {s}")
        assert vn.obs_rms.count == ref.obs_rms.count
        assert vn.ret_rms.mean[0] == ref.ret_rms.mean and vn.ret_rms.var[0] == ref.ret_rms.var
        np.testing.assert_array_equal(vn.returns, ref.returns, err_msg=f"returns {s}")
        assert obs.dtype == np.float32
        np.testing.assert_array_equal(obs, r_obs, err_msg=f"obs {s}")
        np.testing.assert_array_equal(rew, r_rew, err_msg=f"reward {s}")
        for i, t in r_tobs.items():
            saw_done = True
            np.testing.assert_array_equal(infos[i]["terminal_observation"], t)
    assert saw_done
    vn.close()


@pytest.mark.gpu
def test_compact_kernel_occupancy():
    """the main.xml compact tier keeps its working set within 16 KB of LDS (ten would fit a CU) and eight
    envs per CU (two waves per SIMD at <= 256 registers).  Ten envs per CU at 168 registers was built and
    measured slower (occupancy); a change that grows the LDS layout past 20 KB or the register
    count past 256 silently halves throughput"""
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1), 64)
    info = b.kernel_info()
    b.close()
    assert info["lds_bytes"] <= 16384, info
    assert info["envs_per_cu"] >= 8, info


@pytest.mark.gpu
def test_ppo_graph_update_matches_eager():
    """Config C5 driver: the HIP-graph replay of the PPO minibatch update (three eager warm-up
    minibatches, then capture) lands on the same policy as the eager update on the same rollout
    (same seeds, same env): only Adam's device-side bias correction (capturable) rounds
    differently, so parameters agree to 1e-5."""
    torch = _torch()
    from ur3e_amd.envs.vec_env import UR3eVecEnv
    from ur3e_amd.envs.vec_normalize import VecNormalize
    from ur3e_amd.rl.ppo import PPO
    params, stats = [], []
    for graphs in (False, True):
        venv = UR3eVecEnv(num_envs=64, device=0, seed=0)
        env = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=10.0)
        algo = PPO(env, n_steps=4, batch_size=32, n_epochs=2, device="cuda:0", seed=0, graphs=graphs)
        algo.learn(1)
        assert (algo._graphs is not None) == graphs
        params.append(torch.cat([p.detach().reshape(-1) for p in algo.policy.parameters()]).cpu())
        stats.append(algo.stats)
        venv.close()
    d = (params[0] - params[1]).abs().max().item()
    assert d < 1e-5, d
    for k in stats[0]:
        assert abs(stats[0][k] - stats[1][k]) < 1e-4 * max(1.0, abs(stats[0][k])), (k, stats)


def test_sensors_move_l_mug_bit_exact():
    """mjData.sensordata (6 torque via mj_rnePostConstraint, 7 actuatorfrc, 2 touch) on the scripted
    pick (C3 semantics, move_l_mug.py:67-81 records actuator_frc = get_jnt_torques every row): the
    full-capacity kernel's sensordata equals the oracle's bit for bit through the grasp and lift."""
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd.controller.move_l_mug import MoveLMug
    n = 16
    drv = MoveLMug(n, reset_mode="low", seed=5, sensors=True)
    gb = drv.batch
    ob = po.OracleBatch(gb.model_c, _oracle_cfg(po, gb.cfg), n)
    np.testing.assert_array_equal(gb.get_sensordata().cpu().numpy(), ob.sensordata())
    nz_torque = 0
    for s in range(2600):
        row = drv.step()
        ob.step(row.cpu().numpy())
        if s % 100 == 0 or s == 2599:
            torch.cuda.synchronize()
            g = gb.get_sensordata().cpu().numpy()
            o = ob.sensordata()
            np.testing.assert_array_equal(g, o, err_msg=f"sensordata row {s}")
            qp, qv, _ = gb.get_state()
            oqp, oqv, _, _ = ob.get_state()
            np.testing.assert_array_equal(qp.cpu().numpy(), oqp, err_msg=f"qpos row {s}")
            nz_torque += int(np.abs(g[:, :18]).max() > 0)
            af = drv.actuator_frc().cpu().numpy()
            assert af.shape == (n, 7)
    assert nz_torque > 0
    drv.close()


@pytest.mark.parametrize("epb", [0, -64])
def test_sensors_gym_v2(epb):
    """gym ur3e-v2 with sensors on (the handle runs the full-capacity tier): sensordata bit-exact
    every step, including auto-resets (T = 30) and grasp-region contacts"""
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    n = 48
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=13, envs_per_block=epb,
                         max_episode_steps=30, sensors=True)
    gb = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, _oracle_cfg(po, cfg), n)
    rng = np.random.default_rng(13)
    for s in range(80):
        a = _grasp_actions(rng, n, md) if s % 2 else _gym_actions(rng, n, md)
        o = ob.step(a)
        g = gb.step(torch.from_numpy(a))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(g[0].cpu().numpy(), o[0], err_msg=f"obs step {s}")
        np.testing.assert_array_equal(gb.get_sensordata().cpu().numpy(), ob.sensordata(),
                                      err_msg=f"sensordata step {s}")
    gb.close()


def test_sensors_off_refuses_read():
    _torch()
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    gb = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1), 8)
    with pytest.raises(RuntimeError, match="sensors are off"):
        gb.get_sensordata()
    gb.close()
