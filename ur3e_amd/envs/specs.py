"""Per-env-id configuration of the four reference gymnasium envs (register_envs.py:4-25).

Each spec names the step-library task, observation width, action Box, frame_skip,
episode cap and controller gains the reference env uses:

| id | reference | task | obs | action | frame_skip | T | gains |
|---|---|---|---|---|---|---|---|
| ur3e-v0 | ur3e_env.py:23-460 | GYM_V0 | 13 | Box near the mug (ur3e_env.py:94-95) | 2 | 500 (tested before t+=1) | ur3e_env.py gains |
| imitation_indirect-v0 | imitation_env_indirect.py | IMIT_INDIRECT | 24 | v2 Box (:53-54) | 1 | 2500 (before t+=1) | config_l_mug.yml |
| imitation_direct-v0 | imitation_env_direct.py | IMIT_DIRECT | 13 | actuator ctrlrange (:56-58) | 2 | 1200 (before t+=1) | unused |
| ur3e-v2 | ur3e_env2.py | GYM_V2 | 24 | v2 Box (:57-64) | 2 | 2500 (after t+=1) | config_l_mug.yml |

config_l_mug.yml is read when the spec is built (as the reference reads it in each env's __init__,
ur3e_env2.py:66-68), through ur3e_amd.gains: an explicit path, else controller/config/ under the working
directory, else the packaged copy.
"""
from __future__ import annotations

import numpy as np

# x_mug_init, y_mug_init from key "down" (main.xml:416-419): +-0.25 in x/y, z in [0, 0.5], grip in [0, 1]
UR3E_V2_ACTION_LOW = np.array([0.29799994 - 0.25, 0.13349916 - 0.25, 0.0, 0.0])
UR3E_V2_ACTION_HIGH = np.array([0.29799994 + 0.25, 0.13349916 + 0.25, 0.5, 1.0])
# ur3e_env.py:94-95
UR3E_V0_ACTION_LOW = np.array([0.28799994, 0.13349916, 0.005, 0.0])
UR3E_V0_ACTION_HIGH = np.array([0.35799994, 0.35349916, 0.165, 1.0])


def _specs():
    from .. import runtime as rt
    return {
        "gymnasium_env/ur3e-v2": dict(task=rt.TASK_GYM_V2, obs_dim=24, low=UR3E_V2_ACTION_LOW,
                                      high=UR3E_V2_ACTION_HIGH, frame_skip=2, T=2500, gains=rt.GAINS_L_MUG,
                                      trunc_after_increment=True),
        "gymnasium_env/ur3e-v0": dict(task=rt.TASK_GYM_V0, obs_dim=13, low=UR3E_V0_ACTION_LOW,
                                      high=UR3E_V0_ACTION_HIGH, frame_skip=2, T=500, gains=rt.GAINS_V0,
                                      trunc_after_increment=False),
        "gymnasium_env/imitation_indirect-v0": dict(task=rt.TASK_IMIT_INDIRECT, obs_dim=24, low=UR3E_V2_ACTION_LOW,
                                                    high=UR3E_V2_ACTION_HIGH, frame_skip=1, T=2500,
                                                    gains=rt.GAINS_L_MUG, trunc_after_increment=False),
        "gymnasium_env/imitation_direct-v0": dict(task=rt.TASK_IMIT_DIRECT, obs_dim=13, low=None, high=None,
                                                  frame_skip=2, T=1200, gains=rt.GAINS_L_MUG,
                                                  trunc_after_increment=False),
    }


def spec(env_id: str, config_yaml_path: str | None = None) -> dict:
    s = _specs()
    if env_id not in s:
        raise KeyError(env_id)
    d = dict(s[env_id])
    if d["gains"] is not None and env_id != "gymnasium_env/ur3e-v0":  # v0's gains are hard-coded (ur3e_env.py:49-55)
        from .. import gains
        d["gains"] = gains.task_gains(config_yaml_path)
    if d["low"] is None:  # direct torque control: Box = actuator ctrlrange (get_ctrl_ranges)
        from .. import runtime as rt
        md, _ = rt.load_model("main")
        cr = np.asarray(md["act_ctrlrange"], dtype=np.float64)
        d["low"], d["high"] = cr[:, 0].copy(), cr[:, 1].copy()
    return d


ENV_IDS = ("gymnasium_env/ur3e-v0", "gymnasium_env/imitation_indirect-v0", "gymnasium_env/imitation_direct-v0",
           "gymnasium_env/ur3e-v2")
