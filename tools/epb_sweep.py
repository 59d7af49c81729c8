"""Sweep envs_per_block for the fused step kernel (GPU only)."""
import sys, os, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from ur3e_amd import runtime as rt
md, mc = rt.load_model("main")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out = {}
for epb in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "64,16,4,1".split(","))]:
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1, envs_per_block=epb)
    b = rt.Batch(mc, cfg, n)
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
    for i in range(3):
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()
    t = time.perf_counter()
    K = 5
    for i in range(K):
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / K
    out[epb] = dict(ms=dt * 1e3, env_steps_per_s=n / dt)
    print(epb, out[epb], flush=True)
    b.close()
print(json.dumps(out))
