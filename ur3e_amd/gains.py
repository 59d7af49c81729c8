"""Controller gains read from the reference's YAML configs (controller/config/*.yml).

The reference reads its gains at construction, from paths relative to the working directory:
`UR3eEnv2.__init__` reads controller/config/config_l_mug.yml (gymnasium_env/envs/ur3e_env2.py:66-68),
controller/move_l_mug.py:20-27 the same file, controller/move_j.py:46-52 config_j.yml and
controller/move_l.py:92-99 config_l.yml.  The gains are then unpacked positionally --
`kp_pos, kd_pos, ki_pos = pos_gains.values()` (controller/controller_func.py:90-91) and
`kp, kd = gains.values()` (controller_func.py:136) -- so the entries' file order, not their names,
decides which is which, and a section with another number of entries raises ValueError.  This module
does the same.  A path given explicitly wins; otherwise controller/config/<name> under the working
directory is used when it exists (a script run from the reference's checkout, as its own scripts are);
otherwise the copy packaged with ur3e_amd (ur3e_amd/config/, the reference's values).
"""
from __future__ import annotations

import os

import yaml

PACKAGED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config")


def config_path(name: str, path: str | None = None) -> str:
    if path is not None:
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        return path
    cwd = os.path.join("controller", "config", name)
    if os.path.exists(cwd):
        return cwd
    return os.path.join(PACKAGED, name)


def _load(name: str, path: str | None) -> dict:
    with open(config_path(name, path)) as f:
        return yaml.safe_load(f)


def _floats(v, n: int, what: str):
    v = [float(x) for x in v]
    if len(v) != n:  # np.diag(v) @ vec would fail on a mismatched length in the reference
        raise ValueError(f"{what}: expected {n} gains, got {len(v)}")
    return v


def task_gains(path: str | None = None) -> dict:
    """pid_task_ctrl's gains from config_l_mug.yml: {kp_pos, kd_pos, kp_rot, kd_rot} (ki is read, unused)."""
    yml = _load("config_l_mug.yml", path)
    kp_p, kd_p, _ki_p = yml["pos"].values()
    kp_r, kd_r, _ki_r = yml["rot"].values()
    return dict(kp_pos=_floats(kp_p, 3, "pos kp"), kd_pos=_floats(kd_p, 3, "pos kd"),
                kp_rot=_floats(kp_r, 3, "rot kp"), kd_rot=_floats(kd_r, 3, "rot kd"))


def joint_gains(path: str | None = None) -> dict:
    """move_j's pd_joint_ctrl gains from config_j.yml: {kp, kd} (6 each)."""
    yml = _load("config_j.yml", path)
    kp, kd = yml["qpos"].values()
    return dict(kp=_floats(kp, 6, "qpos kp"), kd=_floats(kd, 6, "qpos kd"))


def move_l_gains(path: str | None = None) -> tuple:
    """move_l's two pd_joint_ctrl gain sets from config_l.yml: ({kp, kd} "pos", {kp, kd} "rot")."""
    yml = _load("config_l.yml", path)
    kp_p, kd_p = yml["pos"].values()
    kp_r, kd_r = yml["rot"].values()
    return (dict(kp=_floats(kp_p, 6, "pos kp"), kd=_floats(kd_p, 6, "pos kd")),
            dict(kp=_floats(kp_r, 6, "rot kp"), kd=_floats(kd_r, 6, "rot kd")))


def hold(name: str = "config_l_mug.yml", path: str | None = None) -> int:
    """The trajectory hold count (rows per waypoint) of a config."""
    return int(_load(name, path)["hold"])
