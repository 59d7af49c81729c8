"""Diagnostic: per-stage cycle breakdown of the v2 step kernel (separate -DUR3E_STAGE_TIMING build).
Never quote this build's run time (its atomics serialise lane 0); read the SHARES."""
import ctypes, os, subprocess, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "ur3e_amd", "_lib", "libur3e_amd_timing.so")
if not os.path.exists(LIB):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
                    "-shared", "-Wno-unused-result", "-DUR3E_STAGE_TIMING", "-DW_SMALL_MAXCON=9", "-o", LIB,
                    os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_batch.hip"),
                    os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_vecnorm.hip")], check=True)
os.environ["UR3E_LIB"] = LIB
import torch
from ur3e_amd import runtime as rt
names = {24: "load state+action+carry", 23: "controller / step_pre / reset prep (before each forward)", 0: "kinematics", 1: "com_pos", 2: "crb+copy", 3: "factor_tree(M)", 4: "collision", 5: "make_constraint",
         6: "com_vel", 7: "rne+passive+act", 8: "solve_tree(smooth)", 9: "newton init (eval x2-3, grad)",
         10: "H build", 11: "cholesky / (r) backward solve", 12: "hessian_solve / (r) cholesky",
         18: "(r) forward solve", 19: "(r) ls setup + eval(0)", 20: "(r) ls eval (per call)", 13: "line_search tail", 14: "eval+grad (iter)",
         15: "newton tail", 21: "touch sensors", 22: "badacc check", 16: "euler factor+solve", 17: "integrate", 25: "make_carry", 26: "obs+reward+termination", 27: "commit"}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
epb = int(sys.argv[2]) if len(sys.argv) > 2 else 0
md, mc = rt.load_model("main")
b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1, envs_per_block=epb, schedule=1), n)  # schedule 1: per-env-step kernel (the one with stage marks)
L = rt.load_library()
cyc = (ctypes.c_ulonglong * 32)(); calls = (ctypes.c_ulonglong * 32)()
lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
for i in range(3):
    b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
torch.cuda.synchronize()
L.ur3e_debug_stage_cycles(cyc, calls, 1)
K = 5
for i in range(K):
    b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
torch.cuda.synchronize()
L.ur3e_debug_stage_cycles(cyc, calls, 1)
tot = sum(cyc[k] for k in names)
print(f"per env-substep cycles (lane 0 view), {n} envs, {K} steps")
for k, nm in names.items():
    if calls[k]:
        per = cyc[k] / (n * K * 2)
        print(f"{k:2d} {nm:32s} {per:12.0f} cyc/env-substep  {100.0 * cyc[k] / tot:5.1f}%  calls/env-substep {calls[k] / (n * K * 2):.2f}")
print("total", tot / (n * K * 2))
