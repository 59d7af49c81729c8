"""Single-env gymnasium facade shared by the four reference env classes.

A batch of one env on the GPU through the C ABI; the episode counter and the
truncation test live here so that each facade matches its reference class's
ordering (`ur3e_env2.py` tests t after `t += 1`; `ur3e_env.py:184-194`,
`imitation_env_indirect.py:98-101` and `imitation_env_direct.py:100-103` test it
before). Rendering is out of scope: `render_mode` is accepted and ignored.

Deviation (documented in DESIGN.md): `reset(seed=s)` seeds the counter-based
reset noise (the reference draws it from the global np.random, gym_utils.py:58-59).
"""
from __future__ import annotations

import numpy as np

from .spaces import Box
from .specs import spec


class SingleEnv:
    metadata = {"render_modes": ["human", "rgb_array", "depth_array"], "render_fps": 500}
    ENV_ID = None

    def __init__(self, render_mode=None, device: int = 0, seed: int = 0, config_yaml_path: str | None = None):
        s = spec(self.ENV_ID, config_yaml_path)
        self._spec = s
        self.render_mode = render_mode
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(s["obs_dim"],), dtype=np.float64)
        self.action_space = Box(low=s["low"], high=s["high"], dtype=np.float64)
        self.frame_skip = s["frame_skip"]
        self.dt = 0.001 * self.frame_skip
        self._device = device
        self._seed = seed
        self._batch = None
        self.t = 0

    def _ensure(self, seed=None):
        from .. import runtime as rt
        if self._batch is None or seed is not None:
            if self._batch is not None:
                self._batch.close()
            md, mc = rt.load_model("main")
            cfg = rt.make_config(task=self._spec["task"], frame_skip=self.frame_skip, max_episode_steps=0,
                                 auto_reset=False, model=md, task_gains=self._spec["gains"],
                                 seed=self._seed if seed is None else seed)
            self._batch = rt.Batch(mc, cfg, 1, device=self._device)
            return True
        return False

    def reset(self, *, seed=None, options=None):
        fresh = self._ensure(seed)
        obs = self._batch.obs if fresh else self._batch.reset()
        self.t = 0
        return obs[0].cpu().numpy().copy(), {}

    def step(self, action):
        import torch
        if self._batch is None:
            raise RuntimeError("call reset() before step()")
        a = torch.as_tensor(np.asarray(action, dtype=np.float64).reshape(1, self.action_space.shape[0]))
        obs, rew, term, _, _ = self._batch.step(a)
        T = self._spec["T"]
        if self._spec["trunc_after_increment"]:
            self.t += 1
            truncated = self.t >= T
        else:
            truncated = self.t >= T
            self.t += 1
        return (obs[0].cpu().numpy().copy(), float(rew[0].item()), bool(term[0].item()), bool(truncated), {})

    def render(self):
        return None

    def close(self):
        if self._batch is not None:
            self._batch.close()
            self._batch = None
