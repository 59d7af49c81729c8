"""Stable-Baselines3-compatible batched VecEnv over N GPU-resident UR3e envs.

Replaces `make_vec_env("gymnasium_env/ur3e-v2", n_envs, vec_env_cls=SubprocVecEnv)`
(gymnasium_src/scripts/regular_rl/rl/train_rl.py:38-44): instead of N worker
processes each owning a MuJoCo env and talking over pipes, all N envs live in
HBM and one fused kernel launch steps them all.

API (SB3 VecEnv): num_envs, observation_space, action_space, reset(),
step_async(actions), step_wait() -> (obs, rewards, dones, infos), step(),
close(), get_attr/set_attr/env_method/env_is_wrapped, seed().  infos[i] carries
"terminal_observation" and "TimeLimit.truncated" on episode end (SB3
auto-reset semantics) and "episode" = {r, l, t} like SB3's Monitor wrapper.
`step_torch()` returns device tensors for a torch-ROCm policy (no host copy).
"""
from __future__ import annotations

import time

import numpy as np

from .spaces import Box
from .specs import spec

try:  # subclass SB3's VecEnv when it is installed (it is not in this image)
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _SB3VecEnv
except Exception:  # pragma: no cover
    _SB3VecEnv = object


def _default_stepper(env_id: str, num_envs: int, device: int, seed: int, env_id_offset: int, envs_per_block: int,
                     max_episode_steps: int | None, config_yaml_path: str | None = None):
    """The product stepper: num_envs envs of `env_id` resident on GPU `device` (runtime.Batch)."""
    from .. import runtime as rt
    s = spec(env_id, config_yaml_path)
    md, mc = rt.load_model("main")
    T = s["T"] if max_episode_steps is None else max_episode_steps
    cfg = rt.make_config(task=s["task"], frame_skip=s["frame_skip"], max_episode_steps=T, model=md, seed=seed,
                         env_id_offset=env_id_offset, envs_per_block=envs_per_block, task_gains=s["gains"])
    return rt.Batch(mc, cfg, num_envs, device=device)


class UR3eVecEnv(_SB3VecEnv):
    def __init__(self, num_envs: int = 4096, device: int = 0, seed: int = 0, stepper=None, env_id_offset: int = 0,
                 envs_per_block: int = 0, max_episode_steps: int | None = None,
                 env_id: str = "gymnasium_env/ur3e-v2", render_mode=None, config_yaml_path: str | None = None):
        """`render_mode` is accepted for env_kwargs compatibility (train_rl.py:41 passes "human" when
        config_rl.yml:14 visualize is True) and ignored: rendering is out of scope."""
        s = spec(env_id)
        self.env_id = env_id
        self.num_envs = num_envs
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(s["obs_dim"],), dtype=np.float64)
        self.action_space = Box(low=s["low"], high=s["high"], dtype=np.float64)
        self.render_mode = None
        if stepper is None:
            stepper = _default_stepper(env_id, num_envs, device, seed, env_id_offset, envs_per_block,
                                       max_episode_steps, config_yaml_path)
        if _SB3VecEnv is not object:  # pragma: no cover - SB3 is not installed in this image
            try:  # SB3 2.x: num_envs, spaces, reset_infos, _seeds/_options, render_mode, metadata
                _SB3VecEnv.__init__(self, num_envs, self.observation_space, self.action_space)
            except TypeError:
                pass
        self.stepper = stepper
        self._actions = None
        self._ep_ret = np.zeros(num_envs)
        self._ep_len = np.zeros(num_envs, dtype=np.int64)
        self._t0 = time.time()
        self._attrs = {}

    # -- SB3 VecEnv interface ------------------------------------------------
    def reset(self):
        obs = self.stepper.reset()
        self._ep_ret[:] = 0
        self._ep_len[:] = 0
        return _np(obs)

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        obs, rew, term, trunc, tobs = self.step_torch(self._actions)
        obs = _np(obs)
        rew, dones, infos = self.episode_infos(rew, term, trunc, tobs)
        return obs, rew, dones, infos

    def episode_infos(self, rew, term, trunc, tobs):
        """Host-side SB3 bookkeeping of one step: (rewards, dones, infos) with terminal_observation
        (rows of `tobs` for done envs), TimeLimit.truncated and Monitor's episode {r, l, t}."""
        rew, term, trunc = _np(rew), _np(term).astype(bool), _np(trunc).astype(bool)
        dones = term | trunc
        self._ep_ret += rew
        self._ep_len += 1
        infos = [{} for _ in range(self.num_envs)]
        if dones.any():
            tobs = _np(tobs)
            now = round(time.time() - self._t0, 6)
            for i in np.flatnonzero(dones):
                infos[i]["terminal_observation"] = tobs[i].copy()
                infos[i]["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
                infos[i]["episode"] = {"r": float(self._ep_ret[i]), "l": int(self._ep_len[i]), "t": now}
                self._ep_ret[i] = 0
                self._ep_len[i] = 0
        return rew, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def step_torch(self, actions):
        """Device-tensor step: returns (obs, reward, terminated, truncated, terminal_obs) on the GPU."""
        import torch
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions, dtype=np.float64))
        # no clipping here: like UR3eEnv2.step, actions are used as given (SB3 clips to the Box itself)
        return self.stepper.step(a.reshape(self.num_envs, self.action_space.shape[0]).to(torch.float64))

    def close(self):
        if hasattr(self.stepper, "close"):
            self.stepper.close()

    def seed(self, seed=None):
        return [seed] * self.num_envs

    def get_attr(self, attr_name, indices=None):
        """Per-env attribute values: values stored by set_attr for that env, else the (shared) attribute
        of the batched env.  Raises AttributeError like SB3 for a name that exists nowhere."""
        idx = self._indices(indices)
        per_env = self._attrs.get(attr_name)
        if per_env is None:
            if attr_name == "render_mode":
                return [self.render_mode] * len(idx)
            val = getattr(self, attr_name)
            return [val] * len(idx)
        return [per_env[i] for i in idx]

    def set_attr(self, attr_name, value, indices=None):
        """Store `value` for the selected envs only (SB3 semantics: one value, broadcast to `indices`)."""
        if attr_name not in self._attrs:
            cur = getattr(self, attr_name, None)
            self._attrs[attr_name] = [cur] * self.num_envs
        for i in self._indices(indices):
            self._attrs[attr_name][i] = value

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        """Call a method of the per-env gymnasium facade for the selected envs.  Only the methods a
        batched env can answer per env exist: render (None: rendering is out of scope) and the
        attribute getters; anything else raises AttributeError instead of silently returning None."""
        idx = self._indices(indices)
        if method_name == "render":
            return [None] * len(idx)
        if method_name in ("get_wrapper_attr", "__getattribute__"):
            return [v for v in self.get_attr(method_args[0], idx)]
        raise AttributeError(f"UR3eVecEnv: env_method({method_name!r}) has no per-env meaning on the batched env")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self):
        return [None] * self.num_envs

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return list(indices)


def _np(x):
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)
