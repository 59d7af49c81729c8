"""A/B of the two-tier gym step launch schedules (schedule 2 = substep work queue, 1 = one workgroup
per env-step) at several env counts, same process, same actions; prints env-steps/s per case."""
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
import torch  # noqa: E402

from ur3e_amd import runtime as rt  # noqa: E402

md, mc = rt.load_model("main")
ns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2048,4096,8192").split(",")]
steps, pre = 30, 200
lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
for n in ns:
    gen = torch.Generator(device="cuda")
    gen.manual_seed(n)
    acts = lo + (hi - lo) * torch.rand((pre + steps, n, 4), dtype=torch.float64, device="cuda", generator=gen)
    res = {}
    for rep in range(2):
        for sched in (1, 2):
            b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1234,
                                            schedule=sched), n)
            for i in range(pre):
                b.step(acts[i])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(steps):
                b.step(acts[pre + i])
            e1.record()
            torch.cuda.synchronize()
            v = n * steps / (e0.elapsed_time(e1) * 1e-3)
            res.setdefault(sched, []).append(v)
            b.close()
    print(json.dumps({"n": n, "env_step_launch": res[1], "substep_queue": res[2]}), flush=True)
