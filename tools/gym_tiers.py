"""Diagnostic: per-window tier routing of the gym ur3e-v2 random-action workload (4,096 envs): env-steps
the compact tier bailed, routed straight to the grasp tier, handed on to the full tier, and the contact
histogram of the last step of each window.  usage: gym_tiers.py [n_envs] [steps] [window] [model]"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd import runtime as rt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 600
win = int(sys.argv[3]) if len(sys.argv) > 3 else 50
model = sys.argv[4] if len(sys.argv) > 4 else "main"
md, mc = rt.load_model(model)
b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1), n)
lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
tc0 = b.tier_counts()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for t in range(steps):
    b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
    if (t + 1) % win == 0:
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        tc = b.tier_counts()
        d = [x - y for x, y in zip(tc, tc0)]
        tc0 = tc
        nc = b.get_info()["ncon"].to(torch.int64)
        h = torch.bincount(nc.clamp(max=30), minlength=31).cpu().tolist()
        print(json.dumps({"model": model, "steps": [t + 1 - win, t + 1], "env_steps_per_s": n * win / (ms * 1e-3),
                          "compact_bail_frac": d[0] / (n * win),
                          "grasp_to_full_frac": d[1] / (n * win), "routed_frac": d[2] / (n * win),
                          "ncon_hist": {i: v for i, v in enumerate(h) if v}}), flush=True)
        e0.record()
b.close()
