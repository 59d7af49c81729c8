"""`import register_envs` as the reference scripts do it (register_envs.py:1-25 of derekc22/UR3e):
registers the four gymnasium_env/* ids against the MI355X batched envs and rebinds the calling
script's make_vec_env / VecNormalize so that gymnasium_src SB3 scripts run unchanged (see
ur3e_amd/register_envs.py)."""
from ur3e_amd.register_envs import IDS, REGISTERED, install_drop_in, make, make_vec_env  # noqa: F401

DROP_IN = install_drop_in()
