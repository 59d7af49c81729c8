"""Diagnostic: ms per gym ur3e-v2 env-step (4,096 main.xml envs, 2 substeps) of each kernel layout:
the two-tier default, the per-env-step schedule, the full-capacity tier alone (128 and 64 lanes) and
the compact tier with every env forced to fall back (tier_con_cap).  HIP events on the library stream."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd import runtime as rt  # noqa: E402

VARIANTS = {
    "two_tier_auto": dict(),
    "two_tier_per_env_step": dict(schedule=1),
    "full_tier_128": dict(envs_per_block=-128),
    "full_tier_64": dict(envs_per_block=-64),
    "grasp_tier_cap3": dict(tier_con_cap=3),
    "full_tier_chain_cap-3": dict(tier_con_cap=-3),
}


def main(n=4096, steps=10, only=None):
    md, mc = rt.load_model("main")
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    acts = [lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda", generator=g)
            for _ in range(steps + 3)]
    for name, kw in VARIANTS.items():
        if only and name not in only:
            continue
        b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1, **kw), n)
        for a in acts[:3]:
            b.step(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for a in acts[3:]:
            b.step(a)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        print(json.dumps({"variant": name, "envs": n, "ms_per_step": ms, "env_steps_per_s": n / ms * 1e3,
                          "kernel": b.kernel_info() if hasattr(b, "kernel_info") else None}), flush=True)
        b.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096, only=sys.argv[2].split(",") if len(sys.argv) > 2 else None)
