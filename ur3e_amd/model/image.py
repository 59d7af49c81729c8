"""The MJCF -> ur3e_model_t step and the YAML -> gains step as files, for callers of the C ABI that are not
Python (include/ur3e_batch.h: ur3e_model_from_mjcf, ur3e_config_gains_from_yaml, ur3e_batch_create_from_mjcf).

The library runs these functions through an embedded interpreter (ur3e_amd/csrc/ur3e_mjcf.cpp) and reads
the results back: the model as the raw bytes of ur3e_model_t (the ctypes image of include/ur3e_model.h,
whose layout tests/test_abi.py pins against the C compiler), the gains as 36 little-endian doubles
(task_gains[12], joint_gains[12], rot_joint_gains[12] of ur3e_config_t).  The same functions serve as a
command line for an offline step:

    python -m ur3e_amd.model.image model  path/to/main.xml  main.ur3e [auto|mesh|surrogate]
    python -m ur3e_amd.model.image gains  path/to/config.yml TASK gains.bin
"""
from __future__ import annotations

import struct
import sys


def write_model_image(mjcf_path: str, out_path: str, meshes: str = "auto") -> int:
    """compile_mjcf(mjcf_path) (the reference's MJCF, e.g. assets/main.xml) and write the ur3e_model_t
    bytes; returns their count"""
    from .compiler import compile_mjcf, to_ctypes
    mc = to_ctypes(compile_mjcf(mjcf_path, meshes=meshes or "auto"))
    raw = bytes(mc)
    with open(out_path, "wb") as f:
        f.write(raw)
    return len(raw)


def gains_for_task(task: int, config_yaml_path: str | None) -> tuple:
    """(task_gains[12], joint_gains[12], rot_joint_gains[12]) as the reference reads them for a task:
    config_l_mug.yml's pos/rot PID gains for the task-space tasks (ur3e_env2.py:66-68,
    move_l_mug.py:20-27), config_j.yml for move_j (move_j.py:46-52), config_l.yml's pos/rot joint gains for
    move_l (move_l.py:92-99); ur3e-v0 keeps its hard-coded gains (ur3e_env.py:49-55)."""
    from .. import gains as G
    from .. import runtime as rt
    kw = {}
    if task in (rt.TASK_GYM_V2, rt.TASK_TRAJ_L, rt.TASK_IMIT_INDIRECT, rt.TASK_IMIT_DIRECT):
        kw["task_gains"] = G.task_gains(config_yaml_path)
    elif task == rt.TASK_GYM_V0:
        kw["task_gains"] = rt.GAINS_V0
    c = rt.make_config(task=task, config_yaml_path=config_yaml_path, **kw)
    return list(c.task_gains), list(c.joint_gains), list(c.rot_joint_gains)


def write_gains(config_yaml_path: str | None, task: int, out_path: str) -> None:
    tg, jg, rg = gains_for_task(task, config_yaml_path or None)
    with open(out_path, "wb") as f:
        f.write(struct.pack("<36d", *(tg + jg + rg)))


def main(argv):
    if len(argv) >= 3 and argv[0] == "model":
        n = write_model_image(argv[1], argv[2], argv[3] if len(argv) > 3 else "auto")
        print(f"{argv[2]}: {n} bytes")
    elif len(argv) == 4 and argv[0] == "gains":
        write_gains(argv[1], int(argv[2]), argv[3])
    else:
        print(__doc__)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
