"""Algorithmic FP64 operation count per env-step of the bench workload (bench.py's FP64 roofline).

Runs the flop-counting build of the CPU oracle (oracle/flops: the same C sources with `double` ->
a counting type; +, -, *, / and sqrt each count one) single-threaded on a sample of the bench
workload -- gym ur3e-v2 on main.xml, frame_skip 2, uniform random actions in the v2 Box, 'high'
reset noise -- over the bench's timed window: `pre` env-steps after reset run uncounted, then `steps` are
counted (bench.py times env-steps 505-525 since reset), and writes profiles/flops_rNN.json (main.xml's
box surrogate) or profiles/flops_mesh_rNN.json (main_mesh) with the commit it counted.  The GPU kernels execute the same operations in
the same order (bit-exact parity), so this is also the kernel's algorithmic FP64 work.
usage: python tools/count_flops.py [n_envs] [steps] [round] [pre] [model]"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["OMP_NUM_THREADS"] = "1"


def main(n=64, steps=100, rnd=6, pre=500, model="main", out_path=None):
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "flops"], check=True, stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "libur3e_oracle_flops.so"))
    L.ur3f_get_flops.restype = ctypes.c_ulonglong
    md, mc = rt.load_model(model)
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=0)
    oc = po.config_from(cfg)
    ob = po.OracleBatch(mc, oc, n, L=L)
    # cross-check: the counting build computes the same numbers as the plain oracle
    ref = po.OracleBatch(mc, oc, n)
    rng = np.random.default_rng(0)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    for _ in range(pre):  # the untimed part of the bench window (both builds, so they stay in step)
        a = rng.uniform(lo, hi, size=(n, 4))
        assert np.array_equal(ob.step(a)[0], ref.step(a)[0])
    L.ur3f_reset_flops()
    for _ in range(steps):
        a = rng.uniform(lo, hi, size=(n, 4))
        o1 = ob.step(a)[0]
        o2 = ref.step(a)[0]
        assert np.array_equal(o1, o2)
    total = L.ur3f_get_flops()
    per = total / (n * steps)
    out = {"flops_per_env_step": per, "env_steps": n * steps,
           "sample": f"{n} envs x {steps} gym ur3e-v2 env-steps counted after {pre} uncounted ones since reset "
                     f"(the bench's mid-episode window; main.xml, {model} compile, frame_skip 2, uniform v2-Box actions, "
                     f"'high' reset noise)",
           "model": model, "window_env_steps_since_reset": [pre, pre + steps],
           "counted": "FP64 +, -, *, /, sqrt in the oracle's pipeline (controller, 2 x mj_step, obs/reward); "
                      "comparisons, selects, fabs not counted",
           "source": "tools/count_flops.py over oracle/flops (counting build of oracle/)",
           "head": subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                                  text=True).stdout.strip() or None}
    with open(out_path or os.path.join(
            REPO, "profiles", f"flops{'' if model == 'main' else '_mesh'}_r{rnd:02d}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*(int(x) for x in a[:4]), *a[4:5])
