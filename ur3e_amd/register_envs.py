"""Gymnasium registration mirroring the reference register_envs.py:4-25.

`import ur3e_amd.register_envs` registers "gymnasium_env/ur3e-v2" (and the v0 /
imitation ids, which currently resolve to the same v2 facade — their distinct
epilogues are SURVEY.md §8(f) "next" items) when gymnasium is importable.
"""
ENTRY_V2 = "ur3e_amd.envs.ur3e_env2:UR3eEnv2"
IDS = {
    "gymnasium_env/ur3e-v2": ENTRY_V2,
}

try:  # pragma: no cover - gymnasium is not installed in this image
    from gymnasium.envs.registration import register, registry
    for _id, _entry in IDS.items():
        if _id not in registry:
            register(id=_id, entry_point=_entry)
    REGISTERED = True
except Exception:
    REGISTERED = False


def make(env_id="gymnasium_env/ur3e-v2", **kwargs):
    """gym.make stand-in usable without gymnasium."""
    if env_id not in IDS:
        raise KeyError(env_id)
    from .envs.ur3e_env2 import UR3eEnv2
    return UR3eEnv2(**kwargs)


def make_vec_env(env_id="gymnasium_env/ur3e-v2", n_envs=1, seed=0, env_kwargs=None, vec_env_cls=None, **kwargs):
    """Batched replacement for stable_baselines3.common.env_util.make_vec_env on ur3e-v2."""
    if env_id not in IDS:
        raise KeyError(env_id)
    from .envs.vec_env import UR3eVecEnv
    return UR3eVecEnv(num_envs=n_envs, seed=seed)
