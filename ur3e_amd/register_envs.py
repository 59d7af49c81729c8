"""Gymnasium registration mirroring the reference register_envs.py:4-25.

`import ur3e_amd.register_envs` registers the reference's four ids — ur3e-v0,
imitation_indirect-v0, imitation_direct-v0, ur3e-v2 — against the GPU-backed
facades when gymnasium is importable (it is not in this image; `make` and
`make_vec_env` below work without it).
"""
IDS = {
    "gymnasium_env/ur3e-v0": "ur3e_amd.envs.ur3e_env:UR3eEnv",
    "gymnasium_env/imitation_indirect-v0": "ur3e_amd.envs.imitation_env_indirect:ImitationEnvIndirect",
    "gymnasium_env/imitation_direct-v0": "ur3e_amd.envs.imitation_env_direct:ImitationEnvDirect",
    "gymnasium_env/ur3e-v2": "ur3e_amd.envs.ur3e_env2:UR3eEnv2",
}
ENTRY_V2 = IDS["gymnasium_env/ur3e-v2"]

try:  # pragma: no cover - gymnasium is not installed in this image
    from gymnasium.envs.registration import register, registry
    for _id, _entry in IDS.items():
        if _id not in registry:
            register(id=_id, entry_point=_entry)
    REGISTERED = True
except Exception:
    REGISTERED = False


def _resolve(entry):
    import importlib
    mod, cls = entry.split(":")
    return getattr(importlib.import_module(mod), cls)


def make(env_id="gymnasium_env/ur3e-v2", **kwargs):
    """gym.make stand-in usable without gymnasium."""
    if env_id not in IDS:
        raise KeyError(env_id)
    return _resolve(IDS[env_id])(**kwargs)


def make_vec_env(env_id="gymnasium_env/ur3e-v2", n_envs=1, seed=0, env_kwargs=None, vec_env_cls=None, **kwargs):
    """Batched replacement for stable_baselines3.common.env_util.make_vec_env on any registered id:
    all n_envs live on one GPU and step in one kernel launch (vec_env_cls is ignored)."""
    if env_id not in IDS:
        raise KeyError(env_id)
    from .envs.vec_env import UR3eVecEnv
    kw = dict(env_kwargs or {})
    return UR3eVecEnv(num_envs=n_envs, seed=seed, env_id=env_id, **kw)
