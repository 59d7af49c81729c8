"""Diagnostic: unit timeline of the substep work queue (w_env_step_q), separate -DUR3E_WAVE_TRACE build.
Each (substep, env) unit records when its workgroup pulled it, when its flag wait ended and when it
finished (s_memrealtime, 100 MHz).  Per traced launch this prints the span, the mean unit duration per
substep, the time workgroups spent waiting on flags and between units, and the ideal span (the sum
of unit run times over the resident workgroups), so the launch's overhead can be told from its work.
usage: queue_trace.py [n_envs] [steps]   (UR3E_TRACE_MODEL=main_mesh, UR3E_TRACE_PRE=500: the bench's window)"""
import ctypes, json, os, subprocess, sys
import numpy as np
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
from ur3e_amd import _build
LIB = os.environ.get("UR3E_TRACE_LIB") or _build.TRACE_LIB
if not os.path.exists(LIB):
    _build.build(trace=True)

if __name__ == "__main__":
    product = len(sys.argv) > 4 and sys.argv[4] == "product"  # the product library: steps only, no trace
    if not product:
        os.environ["UR3E_LIB"] = LIB
    import torch
    from ur3e_amd import runtime as rt
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    sched = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    fs = 2
    md, mc = rt.load_model(os.environ.get("UR3E_TRACE_MODEL", "main"))
    b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=fs, model=md, seed=1, schedule=sched), n)
    split = int(os.environ.get("UR3E_SPLIT", "-1"))  # percent of each queue's envs split (default: the library's)
    if split >= 0:
        b.set_queue_split(split)
    print('batch created', flush=True)
    L = rt.load_library()
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
    for i in range(int(os.environ.get("UR3E_TRACE_PRE", "20"))):  # untimed env-steps from reset
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
        torch.cuda.synchronize()
        print("warm-up step", i, flush=True)
    # unit rows sub * n + e, the split units' second halves at fs * n + e; workgroup rows from 12288
    nu = n * (fs + 1)
    nrow = 12288 + 2048
    if product:
        print("product library: warm-up steps ran", flush=True)
        sys.exit(0)
    full = np.zeros((nrow, 4), dtype=np.uint64)
    raws = []
    for i in range(steps):
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
        torch.cuda.synchronize()
        assert L.ur3e_debug_wave_trace(full.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), nrow) == 0
        buf = full[:nu]
        ok = buf[:, 2] > 0
        tp, tr, te = (buf[:, k].astype(np.int64) for k in range(3))
        base = tp[ok].min()
        tp, tr, te = (tp - base) / 100.0, (tr - base) / 100.0, (te - base) / 100.0
        wg = (buf[:, 3] & 0xffffffff).astype(np.int64)
        run, wait = te - tr, tr - tp
        sub = np.arange(nu) // n
        slots = len(np.unique(wg[ok]))
        span = te[ok].max()
        # gaps between a workgroup's consecutive units (queue atomic + LDS reload)
        gaps = []
        first_start, last_end = [], []
        for g in np.unique(wg[ok]):
            idx = np.where(ok & (wg == g))[0]
            o = idx[np.argsort(tp[idx])]
            gaps.extend((tp[o[1:]] - te[o[:-1]]).tolist())
            first_start.append(tp[o[0]]); last_end.append(te[o[-1]])
        last_end = np.array(last_end)
        r = dict(step=i, units=int(ok.sum()), slots=slots, span_us=round(float(span), 1),
                 ideal_span_us=round(float(run[ok].sum() / slots), 1),
                 run_mean_us={int(k): round(float(run[ok & (sub == k)].mean()), 1) for k in range(fs + 1)
                              if (ok & (sub == k)).any()},
                 run_p99_us={int(k): round(float(np.percentile(run[ok & (sub == k)], 99)), 1)
                             for k in range(fs + 1) if (ok & (sub == k)).any()},
                 wait_total_us_per_slot=round(float(wait[ok].sum() / slots), 2),
                 wait_units_gt_1us=int((wait[ok] > 1.0).sum()),
                 gap_mean_us=round(float(np.mean(gaps)), 2) if gaps else None,
                 first_start_max_us=round(float(max(first_start)), 1),
                 slot_end_p10_p50_p90_us=[round(float(np.percentile(last_end, q)), 1) for q in (10, 50, 90)],
                 units_per_slot=[int(x) for x in np.percentile(np.bincount(wg[ok]), [0, 50, 100])])
        print(json.dumps(r), flush=True)
        raws.append(full.copy())
    out = os.environ.get("UR3E_TRACE_OUT")
    if out:
        np.savez_compressed(out, units=np.stack(raws), n=n, fs=fs)
    b.close()
