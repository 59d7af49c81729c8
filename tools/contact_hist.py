"""Diagnostic: contact-count histogram of the C3 scripted pick (move_l_mug) and of the gym ur3e-v2
random-action workload, per trajectory-row window, plus the compact tier's overflow fraction.
Sizes the tiers: the compact tier holds W_SMALL_MAXCON contacts (ur3e_wave.h)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd import runtime as rt  # noqa: E402
from ur3e_amd.controller.move_l_mug import MoveLMug  # noqa: E402


def hist(nc, top=41):
    h = torch.bincount(nc.to(torch.int64).clamp(max=top - 1), minlength=top).cpu().tolist()
    return {i: v for i, v in enumerate(h) if v}


def main(n=4096):
    out = {}
    drv = MoveLMug(n, reset_mode="low", seed=0)
    windows = [(0, 1500), (1500, 1800), (1800, 2100), (2100, 2600), (2600, drv.T)]
    for w0, w1 in windows:
        acc = torch.zeros(41, dtype=torch.int64, device="cuda")
        o0 = drv.batch.overflow_count()
        for t in range(w0, w1):
            drv.batch.step(drv.traj.row(t))
            if t % 10 == 0:
                nc = drv.batch.get_info()["ncon"]
                acc += torch.bincount(nc.to(torch.int64).clamp(max=40), minlength=41)
        torch.cuda.synchronize()
        ov = drv.batch.overflow_count() - o0
        out[f"C3_rows_{w0}_{w1}"] = {"ncon_hist_every10": {i: int(v) for i, v in enumerate(acc.tolist()) if v},
                                     "fallback_frac": ov / float(n * (w1 - w0))}
        print(json.dumps({f"C3_rows_{w0}_{w1}": out[f"C3_rows_{w0}_{w1}"]}), flush=True)
    drv.close()
    md, mc = rt.load_model("main")
    b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1), n)
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
    acc = torch.zeros(41, dtype=torch.int64, device="cuda")
    o0 = b.overflow_count()
    for i in range(1000):
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
        if i % 10 == 0:
            acc += torch.bincount(b.get_info()["ncon"].to(torch.int64).clamp(max=40), minlength=41)
    torch.cuda.synchronize()
    out["gym_v2_1000"] = {"ncon_hist_every10": {i: int(v) for i, v in enumerate(acc.tolist()) if v},
                          "fallback_frac": (b.overflow_count() - o0) / float(n * 1000)}
    print(json.dumps({"gym_v2_1000": out["gym_v2_1000"]}), flush=True)
    b.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
