"""Diagnostic: per-env wave timeline of the v2 step kernel (separate -DUR3E_WAVE_TRACE build).
For each traced launch: launch span (first wave start -> last wave end), per-env duration
distribution, envs that auto-reset inside the step, and the activity profile (how many waves
are still running through the launch), so the tail of a launch can be told from its body.
usage: wave_trace.py [n_envs] [steps]"""
import ctypes, json, os, subprocess, sys
import numpy as np
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "ur3e_amd", "_lib", "libur3e_amd_trace.so")
if not os.path.exists(LIB):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
                    "-shared", "-Wno-unused-result", "-DUR3E_WAVE_TRACE", "-o", LIB,
                    os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_batch.hip"),
                    os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_vecnorm.hip")], check=True)


def simulate(d, order, slots):
    """greedy in-order dispatch of envs (durations d, in `order`) onto `slots` wave slots"""
    import heapq
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for i in order:
        t = heapq.heappop(free) + d[i]
        end = max(end, t)
        heapq.heappush(free, t)
    return round(end, 1)


if __name__ == "__main__":
    os.environ["UR3E_LIB"] = LIB
    import torch
    from ur3e_amd import runtime as rt
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    md, mc = rt.load_model("main")
    b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1), n)
    L = rt.load_library()
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
    for i in range(5):
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
    buf = np.zeros((n, 4), dtype=np.uint64)
    res = []
    prev = None
    for i in range(steps):
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
        torch.cuda.synchronize()
        assert L.ur3e_debug_wave_trace(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), n) == 0
        t0, t1 = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
        base = t0.min()
        s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # us (100 MHz)
        d = e - s
        reset = (buf[:, 3] & 0xff).astype(bool)
        ncon = ((buf[:, 3] >> 8) & 0xff).astype(int)
        span = e.max()
        # activity: waves running at each microsecond
        grid = np.arange(0, span + 1, 1.0)
        active = ((s[None, :] <= grid[:, None]) & (e[None, :] > grid[:, None])).sum(1)
        second = s > np.percentile(s, 40) + 5  # waves that waited for a slot
        r = dict(span_us=float(span), dur_mean=float(d.mean()), dur_p50=float(np.median(d)),
                 dur_p99=float(np.percentile(d, 99)), dur_max=float(d.max()),
                 n_reset=int(reset.sum()), dur_reset_mean=float(d[reset].mean()) if reset.any() else None,
                 round2_frac=float(second.mean()), round1_dur_mean=float(d[~second].mean()),
                 round2_dur_mean=float(d[second].mean()) if second.any() else None,
                 start_last_us=float(s.max()), end_p50_us=float(np.median(e)), end_p99_us=float(np.percentile(e, 99)),
                 active_peak=int(active.max()),
                 us_with_lt_half_peak=float((active < active.max() / 2).sum()),
                 us_with_lt_tenth_peak=float((active < active.max() / 10).sum()),
                 slowest_env=int(d.argmax()), slowest_ncon=int(ncon[d.argmax()]), slowest_reset=bool(reset[d.argmax()]),
                 dur_by_ncon={int(k): round(float(d[ncon == k].mean()), 1) for k in np.unique(ncon)})
        slots = int(active.max())
        r["sim_span_env_order"] = simulate(d, np.arange(n), slots)
        if prev is not None:
            r["corr_prev_step"] = float(np.corrcoef(prev, d)[0, 1])
            r["sim_span_prev_heavy_first"] = simulate(d, np.argsort(-prev, kind="stable"), slots)
        r["sim_span_oracle_heavy_first"] = simulate(d, np.argsort(-d, kind="stable"), slots)
        prev = d
        res.append(r)
        print(json.dumps(r), flush=True)
    b.close()
