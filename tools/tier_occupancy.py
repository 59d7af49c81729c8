"""Diagnostic (GPU): envs resident per CU, LDS bytes and registers of every tier kernel the library picks for the
scripted pick (move_l_mug, TRAJ_L) and the gym ur3e-v2 step, on main and main_mesh.  usage: tier_occupancy.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

if __name__ == "__main__":
    from ur3e_amd import runtime as rt
    for model in ("main", "main_mesh"):
        md, mc = rt.load_model(model)
        for task in (rt.TASK_GYM_V2, rt.TASK_TRAJ_L):
            b = rt.Batch(mc, rt.make_config(task=task, frame_skip=2 if task == rt.TASK_GYM_V2 else 1, model=md,
                                            seed=1), 64)
            for tier in ("step", "mid", "grasp", "full"):
                try:
                    k = b.kernel_info(tier)
                except Exception as ex:  # a build without that tier
                    print(model, task, tier, "n/a", ex)
                    continue
                print(f"{model:10s} task {task} {tier:6s} envs/CU {k['envs_per_cu']:2d} lds {k['lds_bytes']:6d} "
                      f"regs {k['regs']:3d} {k['kernel']}", flush=True)
            b.close()
