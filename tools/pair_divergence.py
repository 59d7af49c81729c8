"""Pair-divergence factor of the compact tier from queue-unit traces (tools/queue_trace.py with
UR3E_TRACE_OUT): if two envs shared one wave64 (32 lanes each), the wave would run until the slower of
the two finished.  Per env-step the run time d = sum over its substep units of (finished - flag
acquired); the factor E[max(d_i, d_j)] / E[d] over pairs (i, j) is the slowdown a packed wave pays
against one env per wave.  Pairs: random (any packing) and neighbours (2k, 2k+1: a static packing).
usage: pair_divergence.py TRACE.npz"""
import json
import sys

import numpy as np

z = np.load(sys.argv[1])
units, n, fs = z["units"], int(z["n"]), int(z["fs"])
rng = np.random.default_rng(0)
res = []
for L in units:  # one traced launch: rows sub * n + e
    u = L[: n * fs].astype(np.int64)
    ok = (u[:, 0] > 0) & (u[:, 1] > 0) & (u[:, 2] >= u[:, 1])
    run = np.where(ok, u[:, 2] - u[:, 1], 0).reshape(fs, n).sum(0) / 100.0  # us (100 MHz stamps)
    good = ok.reshape(fs, n).all(0)
    d = run[good]
    perm = rng.permutation(len(d))
    m = len(d) // 2 * 2
    rand = np.maximum(d[perm[:m:2]], d[perm[1:m:2]]).mean() / d.mean()
    dn = run[: n // 2 * 2].reshape(-1, 2)
    gn = good[: n // 2 * 2].reshape(-1, 2).all(1)
    neigh = dn[gn].max(1).mean() / d.mean()
    res.append(dict(envs=int(good.sum()), mean_us=round(float(d.mean()), 1), p99_us=round(float(np.percentile(d, 99)), 1),
                    factor_random=round(float(rand), 4), factor_neighbours=round(float(neigh), 4)))
print(json.dumps({"launches": res,
                  "factor_random_mean": round(float(np.mean([r["factor_random"] for r in res])), 4),
                  "factor_neighbours_mean": round(float(np.mean([r["factor_neighbours"] for r in res])), 4)}, indent=1))
