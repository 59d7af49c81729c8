"""Algorithmic FP64 operation count per env-step of the bench workload (bench.py's FP64 roofline).

Runs the flop-counting build of the CPU oracle (oracle/flops: the same C sources with `double` ->
a counting type; +, -, *, / and sqrt each count one) single-threaded on a sample of the bench
workload -- gym ur3e-v2 on main.xml, frame_skip 2, uniform random actions in the v2 Box, 'high'
reset noise -- and writes profiles/flops_rNN.json (NN: the round, default 04) with the commit it counted.  The GPU kernels execute the same operations in
the same order (bit-exact parity), so this is also the kernel's algorithmic FP64 work.
usage: python tools/count_flops.py [n_envs] [steps] [round]"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["OMP_NUM_THREADS"] = "1"


def main(n=64, steps=100, rnd=4, out_path=None):
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "flops"], check=True, stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "libur3e_oracle_flops.so"))
    L.ur3f_get_flops.restype = ctypes.c_ulonglong
    md, mc = rt.load_model("main")
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=0)
    oc = po.config_from(cfg)
    ob = po.OracleBatch(mc, oc, n, L=L)
    # cross-check: the counting build computes the same numbers as the plain oracle
    ref = po.OracleBatch(mc, oc, n)
    rng = np.random.default_rng(0)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    L.ur3f_reset_flops()
    for _ in range(steps):
        a = rng.uniform(lo, hi, size=(n, 4))
        o1 = ob.step(a)[0]
        o2 = ref.step(a)[0]
        assert np.array_equal(o1, o2)
    total = L.ur3f_get_flops()
    per = total / (n * steps)
    out = {"flops_per_env_step": per, "env_steps": n * steps,
           "sample": f"{n} envs x {steps} gym ur3e-v2 env-steps (main.xml, frame_skip 2, uniform v2-Box actions, "
                     f"'high' reset noise)",
           "counted": "FP64 +, -, *, /, sqrt in the oracle's pipeline (controller, 2 x mj_step, obs/reward); "
                      "comparisons, selects, fabs not counted",
           "source": "tools/count_flops.py over oracle/flops (counting build of oracle/)",
           "head": subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                                  text=True).stdout.strip() or None}
    with open(out_path or os.path.join(REPO, "profiles", f"flops_r{rnd:02d}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:4]))
