"""Long GPU-vs-oracle rollout (checker, test infrastructure): N gym ur3e-v2 envs x S env-steps of
uniform random actions, crossing the T = 2500 truncation (auto-resets) and every contact / fallback
transition that occurs; compares every obs/reward/done each step and the full state at the end.
usage: python tools/long_parity.py [n_envs] [steps] [model: main | main_mesh]   (prints one JSON line)"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(n=4096, steps=3000, model="main", seed=21):
    import torch
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model(model)
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, max_episode_steps=2500, model=md, seed=seed)
    gb = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(seed)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    first_bad, dones, t0 = None, 0, time.time()
    ovf0 = gb.overflow_count()
    for t in range(steps):
        a = rng.uniform(lo, hi, size=(n, 4))
        o = ob.step(a)
        g = gb.step(torch.from_numpy(a))
        go, gr, gt, gtr = (x.cpu().numpy() for x in g[:4])
        dones += int((o[2] | o[3]).sum())
        same = (np.array_equal(go, o[0]) and np.array_equal(gr, o[1]) and np.array_equal(gt, o[2])
                and np.array_equal(gtr, o[3]))
        if not same and first_bad is None:
            first_bad = t
        if t % 500 == 0:
            print(f"step {t} ok={first_bad is None} dones={dones} {time.time() - t0:.0f}s", file=sys.stderr,
                  flush=True)
    qp, qv, _ = gb.get_state()
    oqp, oqv, _, onc = ob.get_state()
    ncon = gb.get_info()["ncon"].cpu().numpy()
    print(json.dumps(dict(model=model, envs=n, steps=steps, every_step_bit_exact=first_bad is None, first_mismatch_step=first_bad,
                          episodes_ended=dones, fallback_env_steps=int(gb.overflow_count() - ovf0),
                          max_abs_qpos=float(np.abs(qp.cpu().numpy() - oqp).max()),
                          max_abs_qvel=float(np.abs(qv.cpu().numpy() - oqv).max()),
                          ncon_mismatch_envs=int((ncon != onc).sum()))), flush=True)
    gb.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:3]], *sys.argv[3:4])
