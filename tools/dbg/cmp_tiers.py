"""Debug: compact tier (epb 0) vs full tier (epb -128) on identical inputs, field by field."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np
import torch
from ur3e_amd import runtime as rt
md, mc = rt.load_model("main")
n = 64
bs = [rt.Batch(mc, rt.make_config(task=0, frame_skip=2, model=md, seed=7, envs_per_block=e), n) for e in (0, -128)]
rng = np.random.default_rng(7)
lo = np.array([0.04799994, -0.11650084, 0.0, 0.0]); hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
print("reset obs equal", torch.equal(bs[0].obs, bs[1].obs))
print("reset carry equal", torch.equal(bs[0].get_carry(), bs[1].get_carry()))
for s in range(3):
    a = torch.from_numpy(rng.uniform(lo, hi, size=(n, 4)))
    for b in bs:
        b.step(a)
    torch.cuda.synchronize()
    for nm, f in [("qpos", lambda b: b.get_state()[0]), ("qvel", lambda b: b.get_state()[1]),
                  ("warm", lambda b: b.get_state()[2]), ("carry", lambda b: b.get_carry()),
                  ("touch", lambda b: b.get_touch()), ("ctrl", lambda b: b.get_ctrl()), ("obs", lambda b: b.obs)]:
        x, y = f(bs[0]), f(bs[1])
        d = (x != y)
        if d.any():
            idx = torch.nonzero(d.any(dim=1)).flatten()[:5].tolist()
            cols = torch.nonzero(d.any(dim=0)).flatten().tolist()
            print(f"step {s} {nm}: {int(d.any(dim=1).sum())} envs differ, e.g. {idx}, cols {cols[:20]}, "
                  f"max {float((x - y).abs().max()):.3e}")
        else:
            print(f"step {s} {nm}: equal")
