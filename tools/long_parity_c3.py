"""Long GPU-vs-oracle rollout of the C3 scripted pick (checker, test infrastructure): N move_l_mug envs
along build_traj_l_pick_place rows through the grasp and lift, where envs hold 12-20 contacts and
the library routes them to the grasp tier (and switches the pre-pass on and off as the host sees
routing); compares the full state every `every` rows and at the end, and reports the tier counts.
usage: python tools/long_parity_c3.py [n_envs] [rows] [every] [model: main | main_mesh]   (prints one JSON line per check)"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(n=1024, rows=3000, every=250, model="main"):
    import torch
    from oracle import pyoracle as po
    from ur3e_amd.controller.move_l_mug import MoveLMug
    drv = MoveLMug(n, reset_mode="low", seed=7, model=model)
    gb = drv.batch
    ob = po.OracleBatch(gb.model_c, po.config_from(gb.cfg), n)
    t0 = time.time()
    worst = 0.0
    # rows depend on the trajectory only: built up front, so each chunk of `every` GPU steps runs without
    # a synchronisation (the host runs ahead, as in an open-loop rollout)
    all_rows = torch.stack([drv.traj.row(t) for t in range(rows)])
    rows_np = all_rows.cpu().numpy()
    for c0 in range(0, rows, every):
        c1 = min(rows, c0 + every)
        for t in range(c0, c1):
            gb.step(all_rows[t])
        for t in range(c0, c1):
            ob.step(rows_np[t])
        t = c1 - 1
        torch.cuda.synchronize()
        qp, qv, w = (x.cpu().numpy() for x in gb.get_state())
        oqp, oqv, ow, onc = ob.get_state()
        d = max(float(np.abs(qp - oqp).max()), float(np.abs(qv - oqv).max()), float(np.abs(w - ow).max()))
        ncon = gb.get_info()["ncon"].cpu().numpy()
        worst = max(worst, d)
        print(json.dumps({"row": t + 1, "max_abs_state_diff": d, "ncon_mismatch": int((ncon != onc).sum()),
                          "ncon_max": int(ncon.max()), "tiers": list(gb.tier_counts()),
                          "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"model": model, "envs": n, "rows": rows, "bit_exact": worst == 0.0}), flush=True)
    drv.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:4]], *sys.argv[4:5])
