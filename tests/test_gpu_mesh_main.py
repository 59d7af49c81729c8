"""GPU: the reference's full model with convex meshes -- assets/main.xml compiled with synthetic stand-in
hulls for every mesh file it names (tools/make_main_meshes.py -> ur3e_amd/assets/main_mesh.model.json:
24 colliding geoms, 17 of them convex meshes, 234 candidate pairs) -- bit for bit against the oracle.

It runs in the mesh-capable tier set (KSS_NV_M / KSG_NV_M / KSL_M).  The compact and grasp tiers settle
every mesh pair themselves, one pair per wavefront (ur3e_cvx_wave.h: plane-convex, GJK and EPA with the
hull vertices across lanes and the simplex / polytope in LDS); the full-capacity tier runs convex.h per
lane.  Two workloads:
  * gym ur3e-v2 with random actions: no mesh contact, every env-step stays in the compact tier;
  * move_j holding poses where the gripper's linkage meshes rest on the mug and a pad box on the upper
    arm mesh (contacts box-mesh, EPA): with routing (default), with the grasp tier always behind the
    compact one (tier_con_cap 5: no env-step reaches the full-capacity tier), and with a diagnostic
    contact cap (tier_con_cap < 0) sending them to the full-capacity tier -- bit-exact every way."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LO = np.array([0.04799994, -0.11650084, 0.0, 0.0])
HI = np.array([0.54799994, 0.38349916, 0.5, 1.0])


def _cmp(gb, ob, what):
    qp, qv, wa = gb.get_state()
    oqp, oqv, owa, onc = ob.get_state()
    np.testing.assert_array_equal(qp.cpu().numpy(), oqp, err_msg=f"qpos {what}")
    np.testing.assert_array_equal(qv.cpu().numpy(), oqv, err_msg=f"qvel {what}")
    np.testing.assert_array_equal(wa.cpu().numpy(), owa, err_msg=f"warm start {what}")
    np.testing.assert_array_equal(gb.get_info()["ncon"].cpu().numpy(), onc, err_msg=f"ncon {what}")


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_main_mesh_gym_bit_exact_in_the_compact_tier():
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main_mesh")
    assert md["ngeom"] == 24 and int(np.sum(np.asarray(md["geom_type"]) == 7)) == 17
    n, steps = 256, 200
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=21, max_episode_steps=150)
    gb = rt.Batch(mc, cfg, n)
    ki = gb.kernel_info()
    print("kernel", ki)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(3)
    for t in range(steps):
        a = rng.uniform(LO, HI, size=(n, 4))
        o = ob.step(a)
        gb.step(torch.from_numpy(a))
        if t % 20 == 19:
            torch.cuda.synchronize()
            np.testing.assert_array_equal(gb.obs.cpu().numpy(), o[0], err_msg=f"obs step {t}")
            np.testing.assert_array_equal(gb.reward.cpu().numpy(), o[1], err_msg=f"reward step {t}")
            _cmp(gb, ob, f"step {t}")
    tc = gb.tier_counts()
    print("tier counts (compact->grasp, grasp->full, routed):", tc)
    assert tc[1] == 0  # nothing needed EPA: the compact tier settled every mesh pair
    gb.close()


@pytest.mark.parametrize("cap", [0, 5, -1])
def test_main_mesh_contacts_bit_exact(cap):
    torch = _torch()
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main_mesh")
    n, steps = 32, 120
    cfg = rt.make_config(task=rt.TASK_MOVE_J, frame_skip=1, model=md, seed=4, reset_noise=False,
                         reset_key=md["id_key_down"], max_episode_steps=0, auto_reset=False, tier_con_cap=cap)
    gb = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(9)
    q = np.tile(np.array(md["key_qpos"][md["id_key_down"]], float), (n, 1))
    half = n // 2
    q[:half, 1] += rng.uniform(0.36, 0.44, size=half)   # the gripper's linkage meshes on the mug (box)
    q[half:, 3] += rng.uniform(1.15, 1.25, size=n - half)  # a pad box on the upper-arm mesh
    v = np.zeros((n, md["nv"]))
    gb.set_state(q, v)
    ob.set_state(q, v)
    _cmp(gb, ob, "after set_state")
    target = np.concatenate([q[:, :6], np.zeros((n, 1))], axis=1)  # move_j holds the pose
    mesh_contacts = 0
    gt = np.asarray(md["geom_type"])
    for t in range(steps):
        ob.step(target)
        gb.step(torch.from_numpy(target))
        if t % 10 == 9:
            torch.cuda.synchronize()
            _cmp(gb, ob, f"step {t}")
        if t % 30 == 0:
            for i in range(0, n, 4):
                d = po.OracleData(mc)
                qp, qv, _, _ = ob.get_state()
                d.set(qpos=qp[i], qvel=qv[i])
                d.forward()
                c = d.contacts()
                mesh_contacts += sum(int(gt[a] == 7 or gt[b] == 7) for a, b in c["geoms"])
    tc = gb.tier_counts()
    print("tier counts (compact->grasp, grasp->full, routed):", tc, "mesh contacts sampled:", mesh_contacts)
    assert mesh_contacts > 0
    if cap < 0:
        assert tc[1] > 0  # capped: the touching mesh pairs ran GJK + EPA in the full-capacity tier
    elif cap > 0:
        # the grasp tier always behind the compact one (a positive cap): every env-step, touching mesh pairs
        # included, is settled by the wavefront's convex narrowphase in the compact or the grasp tier
        assert tc[1] == 0
    # cap 0 (routing): the compact tier's bails before the host turns routing on (a few steps) go straight to
    # the full-capacity tier, the rest are routed to the grasp tier
    gb.close()
