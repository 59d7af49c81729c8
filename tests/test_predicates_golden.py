"""Task predicates (gym_utils.py:98-172, ur3e_env2.py:230-254) of the oracle vs
golden vectors from the reference run on synthetic contact lists."""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as po


def test_collision_cache_sets(golden, main_model):
    md, _ = main_model
    arm = [b for b in range(md["nbody"]) if (md["mask_arm_bodies"] >> b) & 1]
    grip = [b for b in range(md["nbody"]) if (md["mask_gripper_bodies"] >> b) & 1]
    assert arm == list(golden["cache_arm"])
    assert grip == list(golden["cache_gripper"])


def test_predicates(golden, main_model):
    md, mc = main_model
    L = po.lib()
    for i in range(len(golden["pred_ncon"])):
        nc = int(golden["pred_ncon"][i])
        pairs = golden["pred_pairs"][i][:nc]
        g1 = np.ascontiguousarray(pairs[:, 0], dtype=np.int32)
        g2 = np.ascontiguousarray(pairs[:, 1], dtype=np.int32)
        out = np.zeros(5, np.int32)
        args = [np.ascontiguousarray(golden[k][i], dtype=np.float64) for k in ("pred_tcp", "pred_hnd", "pred_obs")]
        L.ur3o_predicates(ctypes.byref(mc), ctypes.c_int(nc), g1.ctypes.data_as(ctypes.c_void_p),
                          g2.ctypes.data_as(ctypes.c_void_p), *[a.ctypes.data_as(ctypes.c_void_p) for a in args],
                          out.ctypes.data_as(ctypes.c_void_p))
        assert out[0] == golden["pred_grasp"][i], i
        assert out[1] == golden["pred_robust"][i], i
        assert out[2] == golden["pred_selfcol"][i], i
        assert out[3] == golden["pred_toppled"][i], i
        assert out[4] == golden["pred_term"][i], i


def test_v0_epilogue(golden, main_model):
    """ur3e-v0 (gymnasium_env/envs/ur3e_env.py) compute_reward, _check_termination and
    gym_utils.get_table_collision: oracle vs the reference on synthetic contact lists."""
    md, mc = main_model
    for o, a, r, te, tb, pl, nc in zip(golden["v0_obs"], golden["v0_act"], golden["v0_rew"], golden["v0_term"],
                                      golden["v0_table"], golden["v0_pairs"], golden["v0_ncon"]):
        rr, tt, tab = po.v0_epilogue(mc, pl[:nc], o, a)
        assert rr == pytest.approx(r, rel=1e-12, abs=1e-9)
        assert tt == te
        assert tab == tb
