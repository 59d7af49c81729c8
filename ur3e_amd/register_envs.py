"""Gymnasium registration mirroring the reference register_envs.py:4-25, plus the
drop-in hook that lets the reference's SB3 scripts run unchanged.

`import ur3e_amd.register_envs` registers the reference's four ids -- ur3e-v0,
imitation_indirect-v0, imitation_direct-v0, ur3e-v2 -- against the GPU-backed
facades when gymnasium is importable (it is not in this image; `make` and
`make_vec_env` below work without it).

Drop-in (option a).  The reference scripts bind SB3 names
*before* they import the registration module, then fork one process per env:

    from stable_baselines3.common.env_util import make_vec_env      # train_rl.py:6
    from stable_baselines3.common.vec_env import SubprocVecEnv, VecNormalize  # :7
    import register_envs                                              # :9
    venv = make_vec_env(env_id="gymnasium_env/ur3e-v2", n_envs=n_envs,
                        env_kwargs={"render_mode": ...}, vec_env_cls=SubprocVecEnv)  # :38-44
    venv = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=clip_obs)   # :57

The top-level `register_envs.py` of this repository (what `import register_envs`
resolves to when this repository is on the path) calls `install_drop_in()`, which
rebinds `make_vec_env` and `VecNormalize` in the importing module's globals:
`make_vec_env` on a `gymnasium_env/*` id builds one `UR3eVecEnv` (all n_envs
resident on the GPU, one kernel launch per step; `vec_env_cls` is ignored) and
forwards every other id to the original SB3 function; `VecNormalize` over a
`UR3eVecEnv` is the on-device VecNormalize (and `VecNormalize.load` reads its
.npz statistics), any other venv goes to SB3's class.  `render_mode` (config_rl.yml:14
`visualize: True` -> "human") is a no-op.  Other ids and names are left alone.
"""
from __future__ import annotations

import sys

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


def make_vec_env(env_id="gymnasium_env/ur3e-v2", n_envs=1, seed=None, start_index=0, monitor_dir=None,
                 wrapper_class=None, env_kwargs=None, vec_env_cls=None, vec_env_kwargs=None, monitor_kwargs=None,
                 wrapper_kwargs=None, device=0):
    """Batched replacement for stable_baselines3.common.env_util.make_vec_env (same signature) on the
    registered ids: all n_envs live on one GPU and step in one kernel launch.  `vec_env_cls`,
    `monitor_*` and `vec_env_kwargs` have no meaning for a batched env and are ignored (the episode
    statistics Monitor records are in infos[i]["episode"]); a per-env `wrapper_class` cannot wrap a
    batched env and is refused."""
    if env_id not in IDS:
        raise KeyError(env_id)
    if wrapper_class is not None:
        raise NotImplementedError(f"per-env wrapper {wrapper_class!r} over the batched GPU env")
    from .envs.vec_env import UR3eVecEnv
    kw = dict(env_kwargs or {})
    return UR3eVecEnv(num_envs=n_envs, seed=0 if seed is None else int(seed), env_id=env_id,
                      env_id_offset=int(start_index), device=device, **kw)


class _DispatchMakeVecEnv:
    """make_vec_env bound into a script: gymnasium_env/* ids -> make_vec_env above, others -> SB3's."""
    _ur3e = True

    def __init__(self, orig):
        self.orig = orig

    def __call__(self, env_id, *args, **kwargs):
        if isinstance(env_id, str) and env_id in IDS:
            return make_vec_env(env_id, *args, **kwargs)
        return self.orig(env_id, *args, **kwargs)


class _DispatchVecNormalize:
    """VecNormalize bound into a script: over a UR3eVecEnv the on-device VecNormalize (bit-exact SB3
    statistics, ur3e_amd/envs/vec_normalize.py), over anything else the original class."""
    _ur3e = True

    def __init__(self, orig):
        self.orig = orig

    @staticmethod
    def _ours(venv):
        from .envs.vec_env import UR3eVecEnv
        return isinstance(venv, UR3eVecEnv)

    def __call__(self, venv, *args, **kwargs):
        if self._ours(venv):
            from .envs.vec_normalize import VecNormalize
            return VecNormalize(venv, *args, **kwargs)
        return self.orig(venv, *args, **kwargs)

    def load(self, load_path, venv):
        if self._ours(venv):
            from .envs.vec_normalize import VecNormalize
            return VecNormalize.load(load_path, venv)
        return self.orig.load(load_path, venv)

    def __getattr__(self, name):
        return getattr(self.orig, name)


_SKIP_FILES = ("<frozen importlib", "importlib/__init__")


def _importer_globals():
    """Globals of the module whose `import register_envs` is executing (the first frame outside the
    import machinery and the registration modules themselves)."""
    f = sys._getframe(1)
    while f is not None:
        fn = f.f_code.co_filename
        name = f.f_globals.get("__name__", "")
        if not fn.startswith(_SKIP_FILES) and not any(s in fn for s in _SKIP_FILES) and \
                name not in ("register_envs", __name__):
            return f.f_globals
        f = f.f_back
    return vars(sys.modules["__main__"])


def install_drop_in(namespace: dict | None = None) -> dict:
    """Rebind `make_vec_env` / `VecNormalize` in `namespace` (default: the importing module) as the
    module docstring describes.  Returns {name: True} for each name rebound."""
    ns = _importer_globals() if namespace is None else namespace
    done = {}
    mve = ns.get("make_vec_env")
    if mve is not None and not getattr(mve, "_ur3e", False):
        ns["make_vec_env"] = _DispatchMakeVecEnv(mve)
        done["make_vec_env"] = True
    vn = ns.get("VecNormalize")
    if vn is not None and not getattr(vn, "_ur3e", False):
        ns["VecNormalize"] = _DispatchVecNormalize(vn)
        done["VecNormalize"] = True
    return done
