from .ur3e_env2 import UR3eEnv2, UR3E_V2_ACTION_HIGH, UR3E_V2_ACTION_LOW  # noqa: F401
from .ur3e_env import UR3eEnv  # noqa: F401
from .imitation_env_indirect import ImitationEnvIndirect  # noqa: F401
from .imitation_env_direct import ImitationEnvDirect  # noqa: F401
