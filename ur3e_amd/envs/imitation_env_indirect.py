"""Drop-in for `gymnasium_env.envs.imitation_env_indirect:ImitationEnvIndirect`
("gymnasium_env/imitation_indirect-v0", register_envs.py:9-13): v2 action Box through
pid_task_ctrl (config_l_mug gains), 24-d observation, reward -1, never terminates, truncation
at t >= 2500 tested before t += 1, frame_skip 1."""
from .single import SingleEnv


class ImitationEnvIndirect(SingleEnv):
    ENV_ID = "gymnasium_env/imitation_indirect-v0"
