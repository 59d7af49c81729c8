"""Drop-in for `gymnasium_env.envs.imitation_env_direct:ImitationEnvDirect`
("gymnasium_env/imitation_direct-v0", register_envs.py:15-19): actions are raw actuator
controls in the ctrlrange Box (imitation_env_direct.py:56-62), 13-d observation, reward -1,
never terminates, truncation at t >= 1200 tested before t += 1, frame_skip 2.

Deviation: the reference reset_model calls get_init(..., noise_mag=None), which raises
(gym_utils.py noise table); this facade uses the "high" noise of the other envs."""
from .single import SingleEnv


class ImitationEnvDirect(SingleEnv):
    ENV_ID = "gymnasium_env/imitation_direct-v0"
