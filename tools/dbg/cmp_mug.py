"""Debug: MoveLMug compact tier (epb 0) vs full tier (epb -128), first divergent row per env."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
from ur3e_amd.controller.move_l_mug import MoveLMug
n = 16
ds = [MoveLMug(n, reset_mode="low", seed=5, envs_per_block=e) for e in (0, -128)]
first = {}
for t in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2600):
    for d in ds:
        d.step()
    q0, q1 = ds[0].batch.get_state()[0], ds[1].batch.get_state()[0]
    diff = (q0 != q1).any(dim=1)
    for i in torch.nonzero(diff).flatten().tolist():
        if i not in first:
            first[i] = t
            i0, i1 = ds[0].batch.get_info(), ds[1].batch.get_info()
            print(f"env {i} diverges at row {t}: ncon {int(i0['ncon'][i])} vs {int(i1['ncon'][i])}, "
                  f"ovf total {ds[0].batch.overflow_count()}", flush=True)
print("done; diverged envs:", first, "compact-tier overflow env-steps:", ds[0].batch.overflow_count())
