from .ur3e_env2 import UR3eEnv2, UR3E_V2_ACTION_HIGH, UR3E_V2_ACTION_LOW  # noqa: F401
from .vec_env import UR3eVecEnv  # noqa: F401
