"""Sensors (actuatorfrc, torque, touch) of the oracle against laws restated independently.

main.xml declares 6 torque sensors on the arm joint sites, 7 actuatorfrc and 2 touch sensors
(assets/main.xml:384-405); the reference reads the actuatorfrc ones through get_jnt_torques
(utils/utils.py:201-211) after every mj_step of controller/move_l_mug.py (:80).  On the scripted
pick-and-place rollout (C3 semantics) every 100 rows:
  - layout: sensordata follows the declaration order (torque 3 values each, the rest 1);
  - actuatorfrc = the actuator force law written here in numpy: motors clamp(ctrl, ctrlrange) * gear,
    fingers clamp(0.3137255 clamp(ctrl, [0, 255]) - 100 L - 10 L_dot, +-5) with L the 'split'
    tendon 0.5 q_right_driver + 0.5 q_left_driver (main.xml:349-354, :381);
  - torque (mj_rnePostConstraint's cfrc_int at the site, site frame): the sites sit on the joint
    axes, so the component along the joint axis must equal the joint's generalized force that is not
    a contact or connect force -- actuator + passive damping + friction-loss and limit rows -- by the
    Newton-Euler relation cdof' cfrc_int = (M qacc + bias - J_ext' f_ext) at that dof;
  - touch entries equal the touch sensors.
The GPU reproduces the oracle's sensordata bit for bit (tests/test_gpu_parity.py::test_sensors_*).
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def rollout():
    from oracle import pyoracle as po
    from tests.helpers import oracle_pick_place_rows
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    cfg = rt.make_config(task=rt.TASK_TRAJ_L, frame_skip=1, max_episode_steps=0, auto_reset=False,
                         reset_noise="low", reset_key=md["id_key_down"], model=md, seed=5, sensors=True)
    n = 4
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rows = oracle_pick_place_rows(md, mc, ob)
    snaps = []
    for t in range(2600):
        ob.step(np.ascontiguousarray(rows[:, t]))
        if t % 100 == 99:
            qp, qv, wa, nc = ob.get_state()
            snaps.append(dict(sd=ob.sensordata(), ctrl=np.stack([ob.diag(i)["ctrl"][:mc.nu] for i in range(n)]),
                              touch=np.stack([ob.diag(i)["touch"][:mc.ntouch] for i in range(n)])))
    return md, mc, snaps


def test_sensordata_layout(rollout):
    md, mc, snaps = rollout
    assert md["nsensordata"] == 27 and md["nsensor"] == 15
    assert md["sensor_type"][:6] == [2] * 6 and md["sensor_adr"][:7] == [0, 3, 6, 9, 12, 15, 18]
    for sn in snaps:
        assert sn["sd"].shape == (4, 27)


def test_actuatorfrc_law(rollout):
    md, mc, snaps = rollout
    cr = np.array(md["act_ctrlrange"])
    fr = np.array(md["act_forcerange"])
    # arm motors: gain 1, no bias, ctrl clamped to ctrlrange (the ctrl the last step applied)
    adr = {k: md["sensor_adr"][j] for j, k in enumerate(md["sensor_objid"]) if md["sensor_type"][j] == 1}
    for sn in snaps:
        for i in range(4):
            c = sn["ctrl"][i]
            want = np.clip(c[:6], cr[:6, 0], cr[:6, 1]) * np.array(md["act_gear"][:6])
            got = np.array([sn["sd"][i][adr[a]] for a in range(6)])
            np.testing.assert_array_equal(got, want)
            f = sn["sd"][i][adr[6]]
            assert fr[6, 0] <= f <= fr[6, 1]


def test_finger_actuatorfrc_affine_law():
    """fingers_actuator on a chosen state: 0.3137255 ctrl - 100 L - 10 L_dot, clamped to +-5"""
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    q = np.array(md["key_qpos"][md["id_key_down"]], float)
    rng = np.random.default_rng(0)
    adr = [md["sensor_adr"][j] for j in range(md["nsensor"]) if md["sensor_type"][j] == 1 and md["sensor_objid"][j] == 6][0]
    for ctrl6, qd, vd in [(10.0, 0.01, 0.0), (200.0, 0.02, 0.1), (255.0, 0.3, -0.2), (0.0, 0.001, 0.0)]:
        qq = q.copy()
        qq[6] = qd
        qq[10] = qd * 0.5
        v = np.zeros(20)
        v[6], v[10] = vd, vd * 0.25
        d = po.OracleData(mc)
        d.set(qpos=qq, qvel=v, ctrl=np.r_[rng.uniform(-1, 1, 6), ctrl6])
        d.forward()
        L = 0.5 * qq[6] + 0.5 * qq[10]
        Ld = 0.5 * v[6] + 0.5 * v[10]
        want = np.clip(0.3137255 * min(max(ctrl6, 0.0), 255.0) - 100.0 * L - 10.0 * Ld, -5.0, 5.0)
        np.testing.assert_allclose(d.sensordata()[adr], want, rtol=1e-14, atol=1e-14)


def test_torque_axial_component_is_joint_force():
    """random main.xml states (arm moving, mug on the table, gripper contacts possible): the joint-axis
    component of each torque sensor equals actuator + damping + friction-loss/limit force of that dof"""
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    rng = np.random.default_rng(3)
    q0 = np.array(md["key_qpos"][md["id_key_down"]], float)
    cr = np.array(md["act_ctrlrange"])
    tsens = [j for j in range(md["nsensor"]) if md["sensor_type"][j] == 2]
    checked = 0
    for trial in range(40):
        q = q0.copy()
        q[:6] += rng.uniform(-0.4, 0.4, 6)
        v = np.zeros(20)
        v[:6] = rng.uniform(-1, 1, 6)
        ctrl = np.r_[rng.uniform(cr[:6, 0], cr[:6, 1]) * 0.2, rng.uniform(0, 255)]
        d = po.OracleData(mc)
        d.set(qpos=q, qvel=v, ctrl=ctrl)
        d.forward()
        sd, efc = d.sensordata(), d.efc()
        fs = po.forward_state(mc, q, v)
        for j in tsens:
            site = md["sensor_objid"][j]
            body = md["site_bodyid"][site]
            jnt = [k for k in range(md["njnt"]) if md["jnt_bodyid"][k] == body][0]
            dof = md["jnt_dofadr"][jnt]
            R = fs["site_xmat"][site].reshape(3, 3)
            tau_world = R @ sd[md["sensor_adr"][j]:md["sensor_adr"][j] + 3]
            # joint axis in world = body frame axis; the body frame is the site frame here (site at the
            # joint anchor, no site rotation: class force-torque)
            axis = R @ np.array(md["jnt_axis"][jnt])
            act = np.clip(ctrl[dof], cr[dof, 0], cr[dof, 1]) * md["act_gear"][dof]
            passive = -md["dof_damping"][dof] * v[dof]
            rows = (efc["type"] == 1) | (efc["type"] == 3)
            cons = float(efc["J"][rows, dof] @ efc["force"][rows])
            want = act + passive + cons
            np.testing.assert_allclose(axis @ tau_world, want, rtol=1e-9, atol=1e-9 * max(1.0, abs(want)))
            checked += 1
    assert checked == 40 * 6


def test_touch_entries(rollout):
    md, mc, snaps = rollout
    tadr = [md["sensor_adr"][j] for j in range(md["nsensor"]) if md["sensor_type"][j] == 0]
    for sn in snaps:
        np.testing.assert_array_equal(sn["sd"][:, tadr], sn["touch"])
