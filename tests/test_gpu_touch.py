"""GPU: touch sensors with nonzero readings, bit-exact against the oracle (tests/test_touch_states.py
pins the oracle's values against an independent restatement).  The three fixture states -- fish on
the right pad face, on the left pad face (pad = geom A), and left-pad contacts with the pad as
geom B -- are set through ur3e_batch_set_state (forward pass), read through ur3e_batch_get_touch,
then stepped 40 gym ur3e-v2 env-steps with touch, state and contact counts compared every step."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "touch_states.npz")
NAMES = ["right_face", "left_face", "left_geom_b"]


@pytest.mark.parametrize("epb", [0, -128])
def test_touch_nonzero_bit_exact(epb):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    z = np.load(GOLD)
    reps = 4  # each state in several envs (different env ids / workgroups)
    q = np.concatenate([np.tile(z[nm], (reps, 1)) for nm in NAMES])
    v = np.concatenate([np.tile(z[nm + "_qvel"], (reps, 1)) for nm in NAMES])
    n = len(q)
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=5, envs_per_block=epb)
    gb = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    gb.set_state(q, v)
    ob.set_state(q, v)
    gt = gb.get_touch().cpu().numpy()
    ot = np.stack([ob.diag(i)["touch"][:mc.ntouch] for i in range(n)])
    np.testing.assert_array_equal(gt, ot)
    li, ri = gb.touch_index("left"), gb.touch_index("right")
    assert (gt[0:reps, ri] > 0).all() and (gt[reps:2 * reps, li] > 0).all() and (gt[2 * reps:, li] > 0).all()
    rng = np.random.default_rng(0)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    nonzero_steps = 0
    for s in range(40):
        a = rng.uniform(lo, hi, size=(n, 4))
        o = ob.step(a)
        g = gb.step(torch.from_numpy(a))
        torch.cuda.synchronize()
        gt = gb.get_touch().cpu().numpy()
        ot = np.stack([ob.diag(i)["touch"][:mc.ntouch] for i in range(n)])
        np.testing.assert_array_equal(gt, ot, err_msg=f"touch step {s}")
        nonzero_steps += int(gt.max() > 0)
        np.testing.assert_array_equal(g[0].cpu().numpy(), o[0], err_msg=f"obs step {s}")
        qp, qv, _ = gb.get_state()
        oqp, oqv, _, onc = ob.get_state()
        np.testing.assert_array_equal(qp.cpu().numpy(), oqp, err_msg=f"qpos step {s}")
        np.testing.assert_array_equal(qv.cpu().numpy(), oqv, err_msg=f"qvel step {s}")
        np.testing.assert_array_equal(gb.get_info()["ncon"].cpu().numpy(), onc, err_msg=f"ncon step {s}")
    assert nonzero_steps > 0
    gb.close()
