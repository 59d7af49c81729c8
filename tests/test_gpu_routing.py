"""GPU: the host-side routing decision of ur3e_batch_step (grasp-tier pre-pass only while routing is in
use, decided from a host-mapped count that may be up to 16 steps old).

The scripted pick (C3 semantics) is stepped through its grasp rows without synchronising, so the host
runs ahead and the pre-pass is switched on late, and off again, while route hints exist: steps then
run with routing off (the compact tier steps every env and bails what it cannot hold) or on (routed
envs run in the grasp tier beside it).  Routing only moves work between tiers, so the state must stay
bit-exact against the oracle at every check, and routing must actually have happened.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_routing_switches_bit_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import pyoracle as po
    from ur3e_amd.controller.move_l_mug import MoveLMug
    n, rows, every = 256, 2300, 100
    drv = MoveLMug(n, reset_mode="low", seed=11)
    gb = drv.batch
    ob = po.OracleBatch(gb.model_c, po.config_from(gb.cfg), n)
    routed_at = []
    # rows come from the trajectory alone (not from the state), so they are built up front: the GPU
    # loop below then never synchronises inside a chunk and the host runs up to 16 steps ahead
    all_rows = torch.stack([drv.traj.row(t) for t in range(rows)])
    rows_np = all_rows.cpu().numpy()
    for c0 in range(0, rows, every):
        for t in range(c0, c0 + every):
            gb.step(all_rows[t])
        for t in range(c0, c0 + every):
            ob.step(rows_np[t])
        t = c0 + every - 1
        torch.cuda.synchronize()
        qp, qv, w = (x.cpu().numpy() for x in gb.get_state())
        oqp, oqv, ow, onc = ob.get_state()
        assert np.array_equal(qp, oqp) and np.array_equal(qv, oqv) and np.array_equal(w, ow), f"row {t + 1}"
        assert np.array_equal(gb.get_info()["ncon"].cpu().numpy(), onc), f"ncon row {t + 1}"
        routed_at.append(gb.tier_counts()[2] + gb.mid_count())  # routed to the mid or the grasp tier
    assert routed_at[-1] > 0, "the grasp rows never routed an env past the compact tier"
    drv.close()
