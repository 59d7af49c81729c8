"""Touch sensors with a real contact (CPU: the oracle against an independent restatement).

tests/golden/touch_states.npz (tools/make_touch_states.py) holds main.xml states whose pad touch
sensors read > 0: the fish pressed on the right and on the left pad face (pad = geom A of the
pair), and a state whose left-pad contacts have the pad as geom B (the ray is flipped).  Here the
oracle's touch value is checked against mjSENS_TOUCH restated in numpy from the oracle's contacts:
for every contact of the site's body with positive normal force, cast a ray from the contact point
along the contact normal (flipped when the body is geom2) and add the normal force if the ray meets
the site box (MuJoCo 3.3.3 mj_sensorAcc; the sensor sites are main.xml:192,230).  The GPU test
(tests/test_gpu_touch.py) then requires the kernel to reproduce these values bit for bit.
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "touch_states.npz")
CASES = [("right_face", "right", 1), ("left_face", "left", 1), ("left_geom_b", "left", 2)]


def _ray_hits_box(p, d, c, R, half):
    """ray p + t d, t >= 0, against the box (centre c, rotation R, half sizes) -- slab method"""
    lp, ld = R.T @ (p - c), R.T @ d
    t0, t1 = 0.0, np.inf
    for k in range(3):
        if abs(ld[k]) < 1e-15:
            if abs(lp[k]) > half[k]:
                return False
            continue
        a, b = (-half[k] - lp[k]) / ld[k], (half[k] - lp[k]) / ld[k]
        t0, t1 = max(t0, min(a, b)), min(t1, max(a, b))
        if t0 > t1:
            return False
    return True


@pytest.mark.parametrize("name,side,geom_slot", CASES)
def test_touch_state_matches_independent_touch(name, side, geom_slot):
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    z = np.load(GOLD)
    q, v = z[name], z[name + "_qvel"]
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=5)
    ob = po.OracleBatch(mc, po.config_from(cfg), 1)
    ob.set_state(q[None], v[None])
    touch = ob.diag(0)["touch"][:mc.ntouch]
    site = md["id_site_lpad"] if side == "left" else md["id_site_rpad"]
    k = [md["touch_site"][j] for j in range(md["ntouch"])].index(site)
    assert touch[k] > 0
    # independent restatement of mjSENS_TOUCH over the oracle's contacts
    d = po.OracleData(mc)
    d.set(qpos=q, qvel=v)
    d.forward()
    con, efc = d.contacts(), d.efc()
    fs = po.forward_state(mc, q, v)
    sc, sR = fs["site_xpos"][site], fs["site_xmat"][site].reshape(3, 3)
    half = np.array(md["site_size"][site])
    body = md["site_bodyid"][site]
    gb = md["geom_bodyid"]
    total, slots = 0.0, set()
    for i in range(con["n"]):
        b1, b2 = gb[con["geoms"][i][0]], gb[con["geoms"][i][1]]
        if body not in (b1, b2):
            continue
        fn = efc["force"][con["efc_address"][i]]
        if fn <= 0:
            continue
        ray = con["frame"][i][0] * (-1.0 if body == b2 else 1.0)
        if _ray_hits_box(con["pos"][i], ray, sc, sR, half):
            total += fn
            slots.add(2 if body == b2 else 1)
    assert geom_slot in slots  # the intended geom A / geom B case really contributes
    np.testing.assert_allclose(touch[k], total, rtol=1e-12)
