"""Diagnostic: the C3 timed window alone (move_l_mug scripted pick, 4,096 envs, rows 1500..2600 after
the untimed approach), for kernel traces of the tiered step in the grasp regime."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd.controller.move_l_mug import MoveLMug  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g0, g1 = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1500, 2600)
drv = MoveLMug(n, reset_mode="low", seed=0)
for t in range(g0):
    drv.batch.step(drv.traj.row(t))
rows = [drv.traj.row(t) for t in range(g0, g1)]
tc0 = drv.batch.tier_counts()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for r in rows:
    drv.batch.step(r)
e1.record()
torch.cuda.synchronize()
tc = [x - y for x, y in zip(drv.batch.tier_counts(), tc0)]
print(json.dumps({"env_steps_per_s": n * (g1 - g0) / (e0.elapsed_time(e1) * 1e-3), "rows": [g0, g1],
                  "tier_counts": tc}))
