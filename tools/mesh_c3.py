"""Diagnostic: the C3 scripted pick (move_l_mug, controller/move_l_mug.py:67-81) on both compiles of main.xml,
window by window over the trajectory: env-steps/s on the library stream and where the env-steps ran
(compact tier bails, full-capacity tier, routed to the grasp tier).  usage: mesh_c3.py [n_envs] [models]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd.controller.move_l_mug import MoveLMug  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
models = sys.argv[2].split(",") if len(sys.argv) > 2 else ["main_mesh", "main"]
WINDOWS = [(0, 500), (500, 1500), (1500, 1800), (1800, 2100), (2100, 2600), (2600, 3600), (3600, 5000),
           (5000, 7200)]
for model in models:
    drv = MoveLMug(n, reset_mode="low", seed=0, model=model)
    tot_t, tot_steps, tot_tc = 0.0, 0, [0, 0, 0]
    for w0, w1 in WINDOWS:
        w1 = min(w1, drv.T)
        rows = [drv.traj.row(t) for t in range(w0, w1)]
        tc0 = drv.batch.tier_counts()
        m0 = drv.batch.mid_count() if hasattr(drv.batch, "mid_count") else 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in rows:
            drv.batch.step(r)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        tc = [x - y for x, y in zip(drv.batch.tier_counts(), tc0)]
        mid = (drv.batch.mid_count() if hasattr(drv.batch, "mid_count") else 0) - m0
        k = float(n * (w1 - w0))
        tot_t += ms
        tot_steps += w1 - w0
        tot_tc = [a + b for a, b in zip(tot_tc, tc)]
        nc = drv.batch.get_info()["ncon"].to(torch.int64)
        print(json.dumps({"model": model, "rows": [w0, w1], "env_steps_per_s": k / (ms * 1e-3),
                          "compact_bail_frac": tc[0] / k, "full_tier_frac": tc[1] / k, "grasp_routed_frac": tc[2] / k,
                          "mid_routed_frac": mid / k, "ncon_hist_last": {i: v for i, v in enumerate(torch.bincount(nc.clamp(max=40),
                                                                                       minlength=41).tolist()) if v}}),
              flush=True)
    k = float(n * tot_steps)
    print(json.dumps({"model": model, "rows": [0, tot_steps], "env_steps_per_s": k / (tot_t * 1e-3),
                      "compact_bail_frac": tot_tc[0] / k, "full_tier_frac": tot_tc[1] / k,
                      "grasp_routed_frac": tot_tc[2] / k, "summary": True}), flush=True)
    drv.close()
