"""Diagnostic: the C3 scripted pick (box surrogate, 16 envs x 2,600 rows, seed 5 -- tests/test_gpu_c3_record.py's
case) against the oracle every row, per kernel layout: the default tier chain, the full-capacity tier alone
(envs_per_block -128) and the per-env-step compact kernel with its bails forced on (tier_con_cap).  Prints the
first mismatching row and env per layout.  usage: dbg_c3_tiers.py [layout ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(layout, n=16, rows=2600, seed=5):
    import torch
    from oracle import pyoracle as po
    from ur3e_amd.controller.move_l_mug import MoveLMug
    kw = {"default": {}, "full128": {"envs_per_block": -128}, "full64": {"envs_per_block": -64},
          "cap3": {"tier_con_cap": 3}, "capm12": {"tier_con_cap": -12}}[layout]
    drv = MoveLMug(n, reset_mode="low", seed=seed, **kw)
    gb = drv.batch
    ob = po.OracleBatch(gb.model_c, po.config_from(gb.cfg), n)
    traj = torch.stack([drv.traj.row(t) for t in range(rows)])
    bad = None
    for t in range(rows):
        gb.step(traj[t])
        ob.step(traj[t].cpu().numpy())
        torch.cuda.synchronize()
        qp = gb.get_state()[0].cpu().numpy()
        oqp = ob.get_state()[0]
        if not np.array_equal(qp, oqp):
            envs = np.where((qp != oqp).any(axis=1))[0]
            bad = (t, envs.tolist(), float(np.abs(qp - oqp).max()))
            break
    print(layout, "first mismatch (row, envs, max |dq|):", bad, "tiers:", gb.tier_counts(), "mid:", gb.mid_count(),
          flush=True)
    drv.close()
    return bad


if __name__ == "__main__":
    for lay in (sys.argv[1:] or ["default", "full128", "cap3"]):
        run(lay)
