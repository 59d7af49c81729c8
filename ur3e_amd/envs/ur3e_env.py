"""Drop-in for `gymnasium_env.envs.ur3e_env:UR3eEnv` ("gymnasium_env/ur3e-v0",
register_envs.py:4-7): 13-d observation (ur3e_env.py:50-62), the narrow action Box near the
mug (:94-95), pid_task_ctrl with the v0 gains, reward with self/table-collision penalties and
the pick/place termination (ur3e_env.py:240-450), truncation at t >= 500 tested before t += 1."""
from .single import SingleEnv


class UR3eEnv(SingleEnv):
    ENV_ID = "gymnasium_env/ur3e-v0"
