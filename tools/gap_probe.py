"""Diagnostic: the host-side share of a gym env-step at 4,096 envs -- per-step time with (a) no per-step
events, (b) a pair of timing events around every step (bench.py's timed loop), (c) the steps replayed
from a captured HIP graph.  Compare with the queue kernel's own duration (kernel trace).
usage: python tools/gap_probe.py [n_envs] [steps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(n=4096, steps=200):
    import torch
    from ur3e_amd import runtime as rt
    dev = torch.device("cuda:0")
    md, mc = rt.load_model("main")
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, max_episode_steps=2500, model=md, seed=1234)
    b = rt.Batch(mc, cfg, n)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device=dev)
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device=dev)
    acts = lo + (hi - lo) * torch.rand((steps, n, 4), dtype=torch.float64, device=dev, generator=g)
    for t in range(100):
        b.step(acts[t % steps])
    torch.cuda.synchronize()
    out = {}

    def window(tag, per_step_events):
        ev = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(steps):
            if per_step_events:
                a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a0.record()
            b.step(acts[t])
            if per_step_events:
                a1.record()
                ev.append((a0, a1))
        e1.record()
        torch.cuda.synchronize()
        out[tag] = {"us_per_step": e0.elapsed_time(e1) * 1e3 / steps}
        if ev:
            out[tag]["us_inside_step_events"] = sum(x.elapsed_time(y) for x, y in ev) * 1e3 / steps

    window("no_events", False)
    window("step_events", True)
    window("no_events_2", False)
    # (c) HIP graph of K steps over a static action buffer
    K = 10
    static = acts[:K].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for t in range(3):
            b.step(static[t])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for t in range(K):
            b.step(static[t])
    torch.cuda.synchronize()
    reps = steps // K
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    out["graph"] = {"us_per_step": e0.elapsed_time(e1) * 1e3 / (reps * K)}
    window("no_events_3", False)
    print(json.dumps(out, indent=1))
    b.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:3]])
