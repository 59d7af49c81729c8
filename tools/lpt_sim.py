"""Offline model of the substep work queue's launch span (w_env_step_q) under different unit orders, from a
queue trace (tools/queue_trace.py with UR3E_TRACE_OUT: per (substep, env) unit its pull, flag and end times).
Per queue (XCD): 256 resident workgroups, 512 envs x 2 substeps; each workgroup's first unit is static, the
rest are pulled in order by whichever workgroup frees first; a substep-1 unit waits for its env's substep 0.
Unit run times are the traced ones; the pull gap is the traced mean.  Orders compared per traced step t:
  identity        -- the kernel's order (env index);
  prev_desc       -- envs by the previous traced step's run time (both substeps), longest first;
  oracle_desc     -- by this step's own run time (a bound on what any predictor can get).
usage: lpt_sim.py trace.npz"""
import heapq
import sys

import numpy as np


def simulate(run0, run1, order, slots, gap):
    """run0/run1: per-env substep run times (us); order: env order within the queue; returns the span."""
    n = len(order)
    units = [(0, e) for e in order] + [(1, e) for e in order]
    end0 = np.full(n, np.inf)
    free = []  # (time, slot)
    nxt = 0
    span = 0.0
    # static first units
    for s in range(min(slots, n)):
        sub, e = units[nxt]; nxt += 1
        t = run0[e]
        end0[e] = t
        heapq.heappush(free, (t, s))
        span = max(span, t)
    for s in range(min(slots, n), slots):
        heapq.heappush(free, (0.0, s))
    while nxt < len(units):
        t, s = heapq.heappop(free)
        sub, e = units[nxt]; nxt += 1
        t += gap
        if sub == 0:
            t_end = t + run0[e]
            end0[e] = t_end
        else:
            t_end = max(t, end0[e]) + run1[e]
        span = max(span, t_end)
        heapq.heappush(free, (t_end, s))
    return span


def main(path):
    d = np.load(path)
    U, n, fs = d["units"], int(d["n"]), int(d["fs"])
    nq, slots = 8, 256
    nper = n // nq
    runs = []
    for k in range(U.shape[0]):
        b = U[k, : n * fs]
        tr, te = b[:, 1].astype(np.int64), b[:, 2].astype(np.int64)
        ok = b[:, 2] > 0
        run = np.where(ok, (te - tr) / 100.0, 0.0)
        runs.append(run.reshape(fs, n))
        tp = b[:, 0].astype(np.int64)
        span = (te[ok].max() - tp[ok].min()) / 100.0
        print(f"step {k}: traced span {span:.1f} us, routed/absent units {int((~ok).sum())}")
    gap = 0.9
    for k in range(1, len(runs)):
        r0, r1 = runs[k]
        p0, p1 = runs[k - 1]
        res = {}
        for name, key in (("identity", None), ("prev_desc", p0 + p1), ("oracle_desc", r0 + r1),
                          ("prev_sub0_desc", p0)):
            spans = []
            for q in range(nq):
                sl = slice(q * nper, (q + 1) * nper)
                order = np.arange(nper) if key is None else np.argsort(-key[sl], kind="stable")
                spans.append(simulate(r0[sl], r1[sl], order, slots, gap))
            res[name] = max(spans)
        ideal = (r0.sum() + r1.sum()) / (nq * slots)
        corr = np.corrcoef(r0 + r1, p0 + p1)[0, 1]
        print(f"step {k}: ideal {ideal:.1f}  " + "  ".join(f"{a} {v:.1f}" for a, v in res.items()) +
              f"  corr(prev, this) {corr:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
