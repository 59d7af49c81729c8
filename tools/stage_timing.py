"""Diagnostic: per-stage cycle breakdown of the v2 step kernels (separate -DUR3E_STAGE_TIMING build).
Never quote this build's run time (its atomics serialise lane 0); read the SHARES.

usage: stage_timing.py [n_envs] [envs_per_block] [workload: gym | c3] [tier: 0 compact | 1 grasp | 2 full]
       (UR3E_STAGE_MODEL=main_mesh: main.xml with its convex meshes)
  gym: gym ur3e-v2 random actions (2 substeps, per-env-step launch so the stage marks run);
  c3:  the scripted move_l_mug pick (1 substep per row) timed over its grasp rows 1850..2100, where
       routed envs run in the grasp tier."""
import ctypes, os, subprocess, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
# UR3E_TIMING_LIB / UR3E_TIMING_FLAGS: a second diagnostic variant (its own library, extra -D flags)
LIB = os.environ.get("UR3E_TIMING_LIB", os.path.join(REPO, "ur3e_amd", "_lib", "libur3e_amd_timing.so"))
if not os.path.exists(LIB):
    from ur3e_amd import _build  # same flags as the product library (incl. -disable-machine-licm)
    extra = os.environ.get("UR3E_TIMING_FLAGS", "").split()
    subprocess.run([_build.HIPCC] + _build.FLAGS + extra + ["-DUR3E_STAGE_TIMING", "-DW_SMALL_MAXCON=9", "-o", LIB,
                    os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_batch.hip"),
                    os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_vecnorm.hip")], check=True)
os.environ["UR3E_LIB"] = LIB
import torch
from ur3e_amd import runtime as rt
names = {24: "load state+action+carry", 35: "controller (lane 0, substep 0)", 23: "step_pre / reset prep (before each forward)", 0: "kinematics", 1: "com_pos", 2: "crb+copy", 3: "factor_tree(M)", 4: "collision", 5: "make_constraint",
         6: "com_vel", 7: "rne+passive+act", 8: "solve_tree(smooth)", 9: "newton init (eval x2-3, grad)",
         10: "H build", 11: "cholesky / (r) backward solve", 12: "hessian_solve / (r) cholesky",
         18: "(r) forward solve", 19: "(r) ls setup + eval(0)", 20: "(r) ls eval (per call)", 13: "line_search tail", 14: "eval+grad (iter)",
         15: "newton tail", 21: "touch sensors", 22: "badacc check", 16: "euler factor+solve", 17: "integrate", 25: "make_carry", 26: "obs+reward+termination", 27: "commit",
         28: "(count only) block-diagonal Newton directions", 29: "(r) kinematics: orientation level chain",
         30: "(r) kinematics: position level chain", 31: "(r) com_vel: cvel level chain",
         32: "(r) com_pos: subtree com sums", 33: "(r) com_pos: cdof", 34: "(r) crb: composite inertia sums",
         36: "(r) constraint rows: layout", 37: "(r) constraint rows: group data", 38: "(r) constraint rows: Jacobian",
         39: "(r) collision: broadphase", 40: "(r) tree LDL' factor (smooth + Euler)",
         41: "(r) eval: J.qacc, M.qacc", 42: "(r) eval: constraint update", 43: "(r) eval: cost sums",
         44: "(r) grad: J'f", 45: "(r) ls eval: row terms", 46: "(r) ls eval: sums", 47: "(r) direction: cone Hessians",
         48: "(r) collision: mesh pairs (wave GJK/EPA)", 49: "(count only) mesh pairs settled by the wave"}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
epb = int(sys.argv[2]) if len(sys.argv) > 2 else 0
work = sys.argv[3] if len(sys.argv) > 3 else "gym"
tier = int(sys.argv[4]) if len(sys.argv) > 4 else 0
L = rt.load_library()
L.ur3e_debug_stage_cycles_tier.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
cyc = (ctypes.c_ulonglong * 50)(); calls = (ctypes.c_ulonglong * 50)()
MODEL = os.environ.get("UR3E_STAGE_MODEL", "main")  # main | main_mesh
if work == "gym":
    md, mc = rt.load_model(MODEL)
    # schedule 1: the per-env-step kernel (the one with stage marks)
    b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1, envs_per_block=epb,
                                    schedule=1), n)
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device="cuda")
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device="cuda")
    for i in range(int(os.environ.get("UR3E_STAGE_PRE", "3"))):  # untimed env-steps from reset first
        b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))
    K, subs = 5, 2
    steps = [lambda: b.step(lo + (hi - lo) * torch.rand((n, 4), dtype=torch.float64, device="cuda"))] * K
else:
    from ur3e_amd.controller.move_l_mug import MoveLMug
    drv = MoveLMug(n, reset_mode="low", seed=0, model=MODEL)
    b = drv.batch
    r0, K, subs = 1850, 250, 1
    for t in range(r0):
        b.step(drv.traj.row(t))
    steps = [(lambda t=t: b.step(drv.traj.row(t))) for t in range(r0, r0 + K)]
torch.cuda.synchronize()
L.ur3e_debug_stage_cycles_tier(tier, cyc, calls, 1)
for f in steps:
    f()
torch.cuda.synchronize()
L.ur3e_debug_stage_cycles_tier(tier, cyc, calls, 1)
tot = sum(cyc[k] for k in names if k not in (28, 49))
units = calls[23] if calls[23] else 1  # forward passes run (substeps + retries + resets)
print(f"tier {tier}, workload {work}: per-forward cycles (lane 0 view), {n} envs, {K} steps, "
      f"{calls[23]} forward passes in this tier")
for k, nm in names.items():
    if calls[k]:
        per = cyc[k] / units
        print(f"{k:2d} {nm:32s} {per:12.0f} cyc/forward  {100.0 * cyc[k] / tot:5.1f}%  calls/forward {calls[k] / units:.2f}")
print("total per forward", tot / units)
