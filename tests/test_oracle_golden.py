"""Pin the CPU oracle against golden vectors generated from the reference Python
(tools/make_golden.py; controller_func.py, move_j.py, move_l.py, ur3e_env2.py,
gym_utils.py run with stub mujoco/gymnasium modules)."""
import numpy as np
import pytest

from oracle import pyoracle as po


def test_rot_err(golden):
    for xm, t, e in zip(golden["rot_xmat"], golden["rot_target"], golden["rot_err"]):
        np.testing.assert_allclose(po.rot_err(xm, t), e, rtol=0, atol=1e-12)


def test_pid_task_ctrl(golden):
    gains = [220, 220, 120, 20, 20, 40, 35, 15, 15, 2, 2, 2]  # config_l_mug.yml
    for i in range(len(golden["pid_ctrl"])):
        u = po.pid_task_ctrl_raw(golden["pid_traj"][i], golden["pid_xpos"][i], golden["pid_xmat"][i],
                                 golden["pid_jac"][i], golden["pid_qvel"][i], golden["pid_bias"][i], gains)
        np.testing.assert_allclose(u, golden["pid_ctrl"][i], rtol=1e-12, atol=1e-10)


def test_move_j(golden):
    kp = np.array([20.0, 380.0, 300.0, 20.0, 30.0, 10.0])
    kd = np.full(6, 5.0)
    jr = golden["movej_jnt_range"].reshape(12)
    cr = golden["movej_ctrl_range"][:6].reshape(12)
    for i in range(len(golden["movej_u"])):
        q, v, tgt = golden["movej_q"][i], golden["movej_v"][i], golden["movej_target"][i]
        u = po.pd_joint_ctrl_raw(q, v, tgt[:6] - q, jr, cr, kp, kd)
        np.testing.assert_array_equal(u, golden["movej_u"][i][:6])
        assert golden["movej_u"][i][6] == tgt[6] * 255.0


def test_pinv(golden):
    for J, P in zip(golden["movel_jacp"], golden["movel_pinvp"]):
        np.testing.assert_allclose(po.pinv3x6(J), P, rtol=1e-9, atol=1e-12)


def test_move_l_ctrl(golden):
    """move_l.ctrl (controller/move_l.py:15-78) on synthetic MjData: the oracle's normal-equation
    pinv (the formula the HIP kernel evaluates bit-identically) vs the reference's np.linalg.pinv (SVD)."""
    jr = golden["movej_jnt_range"].reshape(12)
    cr = golden["movej_ctrl_range"][:6].reshape(12)
    pos, rot = golden["cfgl_pos"], golden["cfgl_rot"]
    for i in range(len(golden["movel_u"])):
        u = po.move_l_ctrl_raw(golden["movel_traj"][i], golden["movel_xpos"][i], golden["movel_xmat"][i],
                               golden["movel_jacp"][i], golden["movel_jacr"][i], golden["movel_q"][i],
                               golden["movel_v"][i], jr, cr, pos[0], pos[1], rot[0], rot[1])
        np.testing.assert_allclose(u, golden["movel_u"][i], rtol=1e-9, atol=1e-9)


def test_reward(golden):
    for o, a, r in zip(golden["rew_obs"], golden["rew_act"], golden["rew"]):
        assert po.reward_v2(o, a) == pytest.approx(r, rel=1e-13, abs=1e-13)
    # SURVEY.md Appendix B known answer
    assert golden["rew"][-1] == pytest.approx(7.814356817606531, rel=1e-15)


def test_philox_kat():
    assert po.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert po.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert po.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_tcp_known_answer(main_model):
    md, mc = main_model
    f = po.forward_state(mc, np.array(md["key_qpos"][md["id_key_down"]]))
    # main.xml:415 comment: tcp at 'down' = (0.29799994, 0.13349916, 0.1682003)
    np.testing.assert_allclose(f["site_xpos"][md["id_site_tcp"]], [0.29799994, 0.13349916, 0.1682003], atol=5e-9)
    # ur3e_env2.py:74 target rotation = tcp rotvec at 'down' (~ -1.209, -1.209, 1.209)
    rv = -po.rot_err(f["site_xmat"][md["id_site_tcp"]], np.zeros(3))
    np.testing.assert_allclose(rv, [-1.2092, -1.2092, 1.2092], atol=2e-4)
