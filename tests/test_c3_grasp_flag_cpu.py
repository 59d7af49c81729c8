"""CPU (oracle only): why the scripted pick's grasp flag stays 0 on main.xml (BENCH C3 recording leg:
grasp_rows_recorded_frac 0).  get_task_space_state's flag (controller_func.py:191-200, utils/utils.py:238-245)
compares the pad touch sensors lexicographically with (0.1, 0.1); a touch sensor (main.xml:402-404) sums the
normal forces of contacts whose point lies inside its site box, right/left_pad1_site (main.xml:192, :230:
half sizes 0.01 x 0.0005 x 0.017 about pos (0, -0.007, 0.018125) in the pad body).  The pads are the
reference's own boxes (main.xml:81-88: pad_box1 half sizes 0.011 x 0.004 x 0.009375), not surrogates.

In the grasp window every pad1-mug contact the box-box narrowphase emits sits on a corner of the pad box:
|x| = 0.011 (the pad's half width, beyond the site's 0.01) at the pad's top edge (z = 0.01 + 0.009375 =
0.019375 in the site frame, beyond the site's 0.017) -- the mug meets the pad's top edge, not its face -- so
no contact point is inside a touch site, both touch readings are 0 and the flag is 0.  Pinned here on the
oracle's contact positions, expressed in the site frames from the oracle's kinematics."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def test_pad_contacts_lie_on_pad_corners_outside_the_touch_sites():
    from helpers import oracle_pick_place_rows
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    cfg = rt.make_config(task=rt.TASK_TRAJ_L, frame_skip=1, max_episode_steps=0, auto_reset=False, reset_noise=3,
                         reset_key=md["id_key_down"], model=md, seed=0)
    n = 4
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rows = oracle_pick_place_rows(md, mc, ob)
    gn, sn = md["geom_names"], md["site_names"]
    pads = {gn.index("right_pad1"): sn.index("right_pad1_site"), gn.index("left_pad1"): sn.index("left_pad1_site")}
    fish = gn.index("fish")
    half = np.array([0.01, 0.0005, 0.017])  # the sites' box half sizes (main.xml:192, :230)
    seen = 0
    for t in range(2600):
        ob.step(rows[:, t])
        if t < 1700 or t % 100:
            continue
        qp, qv, _, _ = ob.get_state()
        for i in range(n):
            fs = po.forward_state(mc, qp[i], qv[i])
            d = po.OracleData(mc)
            d.set(qpos=qp[i], qvel=qv[i])
            d.forward()
            c = d.contacts()
            for k, (a, b) in enumerate(c["geoms"]):
                for g in (a, b):
                    if g not in pads or fish not in (a, b):
                        continue
                    s = pads[g]
                    R = np.asarray(fs["site_xmat"][s]).reshape(3, 3)
                    loc = R.T @ (c["pos"][k] - np.asarray(fs["site_xpos"][s]))
                    seen += 1
                    assert (np.abs(loc) > half).any(), (t, i, gn[g], loc)  # outside the touch site
                    # on the pad box's corner: the half width and the top edge
                    np.testing.assert_allclose(abs(loc[0]), 0.011, atol=2e-5)
                    np.testing.assert_allclose(loc[2], 0.019375, atol=1e-4)
            touch = ob.diag(i)["touch"]
            assert touch[0] == 0 and touch[1] == 0
        st = ob.task_space_state(1, 0)  # touch columns: right_pad1_contact, left_pad1_contact (main.xml:402-404)
        assert (st[:, 6] == 0).all()
    assert seen >= 20  # the pads do touch the mug in this window
