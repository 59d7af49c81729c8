"""Drop-in for `gymnasium_env.envs.ur3e_env2:UR3eEnv2` ("gymnasium_env/ur3e-v2",
register_envs.py:22-25): Box(-inf, inf, (24,), f64) observations (ur3e_env2.py:44-48),
the Box around the `down` mug position as action space (ur3e_env2.py:57-64),
render_fps 500, frame_skip 2, truncation at t >= 2500 after the increment.  The physics
runs on the GPU through the C ABI; there is no CPU path."""
from .single import SingleEnv
from .specs import UR3E_V2_ACTION_HIGH, UR3E_V2_ACTION_LOW  # noqa: F401  (re-exported)


class UR3eEnv2(SingleEnv):
    ENV_ID = "gymnasium_env/ur3e-v2"
