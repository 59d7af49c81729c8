"""Diagnostic: cycles of single compact-tier stages, each repeated on primed per-env LDS state
(-DUR3E_STAGE_TIMING build, ur3e_debug_stage_bench).  usage: stage_bench.py [n_envs] [reps]"""
import ctypes, os, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "ur3e_amd", "_lib", "libur3e_amd_timing.so")
os.environ["UR3E_LIB"] = LIB
import torch
from ur3e_amd import runtime as rt
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
md, mc = rt.load_model("main")
b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1, envs_per_block=0), n)
L = rt.load_library()
lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
for i in range(20):
    b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
torch.cuda.synchronize()
names = ["kinematics", "com_pos", "crb", "collision", "make_constraint", "vel_acc", "rne_passive",
         "tree_solve", "solve_newton", "forward(all)", "kin: preload only", "kin: levels copy-only",
         "kin: no frames", "mc: layout only", "mc: +phase A (J)", "mc: +phase B (aref,R)", "coll: count pass"]
only = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
cyc = torch.zeros(n, dtype=torch.int64, device="cuda")
L.ur3e_debug_stage_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
for st, nm in enumerate(names):
    if only is not None and st not in only:
        continue
    rc = L.ur3e_debug_stage_bench(b.h, st, reps, ctypes.c_void_p(cyc.data_ptr()))
    assert rc == 0
    c = cyc[cyc > 0].double()
    print(f"{st:2d} {nm:16s} mean {c.mean().item():9.0f}  median {c.median().item():9.0f} cycles/call  (n={c.numel()})",
          flush=True)
