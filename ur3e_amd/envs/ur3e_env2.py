"""Single-env gymnasium facade with the reference `UR3eEnv2` API.

Drop-in for `gymnasium_env.envs.ur3e_env2:UR3eEnv2` (registered as
"gymnasium_env/ur3e-v2", register_envs.py:22-25): same observation space
(Box(-inf, inf, (24,), float64), ur3e_env2.py:44-48), same action space
(Box around the `down` mug position, ur3e_env2.py:57-64), same metadata
(render_fps 500), same reset()/step() return shapes.  The physics runs on the
GPU through the C ABI (a batch of one env); there is no CPU path.

Deviation (documented in DESIGN.md): `reset(seed=s)` seeds the counter-based
mug-position noise (the reference draws it from the global np.random and
ignores the seed, gym_utils.py:58-59).
"""
from __future__ import annotations

import numpy as np

from .spaces import Box

# x_mug_init, y_mug_init from key "down" (main.xml:416-419): +-0.25 in x/y, z in [0, 0.5], grip in [0, 1]
UR3E_V2_ACTION_LOW = np.array([0.29799994 - 0.25, 0.13349916 - 0.25, 0.0, 0.0])
UR3E_V2_ACTION_HIGH = np.array([0.29799994 + 0.25, 0.13349916 + 0.25, 0.5, 1.0])


class UR3eEnv2:
    metadata = {"render_modes": ["human", "rgb_array", "depth_array"], "render_fps": 500}

    def __init__(self, render_mode=None, device: int = 0, seed: int = 0):
        self.render_mode = render_mode  # rendering is out of scope: accepted and ignored
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(24,), dtype=np.float64)
        self.action_space = Box(low=UR3E_V2_ACTION_LOW, high=UR3E_V2_ACTION_HIGH, dtype=np.float64)
        self.frame_skip = 2
        self.dt = 0.002
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
            cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, max_episode_steps=0, auto_reset=False,
                                 model=md, seed=self._seed if seed is None else seed)
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
        a = torch.as_tensor(np.asarray(action, dtype=np.float64).reshape(1, 4))
        obs, rew, term, trunc, _ = self._batch.step(a)
        self.t += 1
        truncated = self.t >= 2500
        return (obs[0].cpu().numpy().copy(), float(rew[0].item()), bool(term[0].item()), bool(truncated), {})

    def render(self):
        return None

    def close(self):
        if self._batch is not None:
            self._batch.close()
            self._batch = None
