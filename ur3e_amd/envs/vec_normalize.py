"""SB3 `VecNormalize` kept on the GPU (include/ur3e_vecnorm.h).

Replaces `VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=clip_obs)`
(gymnasium_src/scripts/regular_rl/rl/train_rl.py:57) around the batched env: the running
observation statistics, the discounted returns and their statistics live in HBM and are updated by
the library's kernels right after each step, in numpy's reduction order, so `obs_rms` / `ret_rms`
match SB3 (stable_baselines3==2.7.0) bit-for-bit on the same inputs.  `step_torch` hands the
normalised float32 observations to a torch-ROCm policy without a host copy; `step_wait` keeps the
SB3 VecEnv contract (numpy obs, rewards, dones, infos with the normalised terminal observation).

Several ranks (one process per GPU, each stepping its own env shard): pass the
process group.  SB3 keeps ONE RunningMeanStd over all envs of the VecEnv, so each step every rank
all-gathers the shard outputs (one collective, rank-major = global env-id order) and runs the same
statistics kernel over the whole global batch: the statistics, the per-env discounted returns and the
normalised outputs are then identical on every rank and identical to a single-process VecNormalize over
all envs; each rank keeps its own rows.

Persistence: `save(path)` / `VecNormalize.load(path, venv)` write the statistics and settings as an
.npz archive at exactly `path`, whatever its suffix (train_rl.py:20,90 save to `rl_vecnormalize_*.pkl`
and :49 / evaluate_rl.py:30 load that same name; SB3 pickles the wrapper object, its fields are the same).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import runtime as rt


STATS_KEYS = ("obs_mean", "obs_var", "obs_count", "ret_mean", "ret_var", "ret_count", "cfg")


def write_stats(path, **arrays):
    """np.savez into exactly `path` (whatever its suffix)."""
    missing = set(STATS_KEYS) - set(arrays)
    if missing:
        raise ValueError(f"VecNormalize statistics lack {sorted(missing)}")
    with open(path, "wb") as f:
        np.savez(f, **arrays)


def read_stats(path) -> dict:
    """The arrays write_stats() stored at `path`.  A file saved by an older build of this package at
    `path + '.npz'` (np.savez's suffix) is read too.  Anything that is not such an .npz raises."""
    import os
    import zipfile
    p = str(path)
    if not os.path.exists(p) and os.path.exists(p + ".npz"):
        p = p + ".npz"
    if not os.path.exists(p):
        raise FileNotFoundError(f"no VecNormalize statistics at {path!r}")
    if not zipfile.is_zipfile(p):
        raise ValueError(f"{p!r} is not a VecNormalize .npz written by ur3e_amd (SB3 pickles are not "
                         "loaded: re-save the statistics with VecNormalize.save from this package)")
    with np.load(p) as z:  # allow_pickle=False
        out = {k: z[k] for k in z.files}
    missing = set(STATS_KEYS) - set(out)
    if missing:
        raise ValueError(f"{p!r} lacks VecNormalize fields {sorted(missing)}")
    return out


class StatsC(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in ("obs_mean", "obs_var", "obs_count", "ret_mean", "ret_var",
                                                "ret_count", "returns")]


class CfgC(ctypes.Structure):
    _fields_ = [("training", ctypes.c_int), ("norm_obs", ctypes.c_int), ("norm_reward", ctypes.c_int),
                ("clip_obs", ctypes.c_double), ("clip_reward", ctypes.c_double), ("gamma", ctypes.c_double),
                ("epsilon", ctypes.c_double)]


def _bind(L):
    vp, ip = ctypes.c_void_p, ctypes.c_int
    L.ur3e_vecnorm_step.argtypes = [vp, vp, ip, ip, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.ur3e_vecnorm_reset.argtypes = [vp, vp, ip, ip, vp, vp, vp]
    L.ur3e_vecnorm_normalize_obs.argtypes = [vp, vp, ip, ip, vp, vp, vp]
    return L


class _RMSView:
    """obs_rms / ret_rms with SB3's attribute names (host copies of the device statistics)."""

    def __init__(self, mean, var, count):
        self._m, self._v, self._c = mean, var, count

    @property
    def mean(self):
        return self._m.cpu().numpy().copy()

    @property
    def var(self):
        return self._v.cpu().numpy().copy()

    @property
    def count(self):
        return float(self._c.item())


class VecNormalize:
    def __init__(self, venv, training: bool = True, norm_obs: bool = True, norm_reward: bool = True,
                 clip_obs: float = 10.0, clip_reward: float = 10.0, gamma: float = 0.99, epsilon: float = 1e-8,
                 group=None):
        import torch
        self.torch = torch
        self.venv = venv
        self.num_envs = venv.num_envs
        # statistics run over every rank's envs (global env-id order); this rank owns rows [lo, lo + n)
        self.group = group
        if group is not None:
            import torch.distributed as dist
            self._world, self._rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            self._world, self._rank = 1, 0
        self.n_stats = self.num_envs * self._world
        self.observation_space = venv.observation_space
        self.action_space = venv.action_space
        self.render_mode = getattr(venv, "render_mode", None)
        self.L = _bind(rt.load_library())
        dev = venv.stepper.device
        self.device = dev
        dim = self.observation_space.shape[0]
        self.dim = dim
        f64 = dict(dtype=torch.float64, device=dev)
        # RunningMeanStd(epsilon=1e-4): mean 0, var 1, count 1e-4
        self._obs_mean = torch.zeros(dim, **f64)
        self._obs_var = torch.ones(dim, **f64)
        self._obs_count = torch.full((1,), 1e-4, **f64)
        self._ret_mean = torch.zeros(1, **f64)
        self._ret_var = torch.ones(1, **f64)
        self._ret_count = torch.full((1,), 1e-4, **f64)
        self._returns = torch.zeros(self.n_stats, **f64)
        self._st = StatsC(*[t.data_ptr() for t in (self._obs_mean, self._obs_var, self._obs_count, self._ret_mean,
                                                     self._ret_var, self._ret_count, self._returns)])
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon
        self._obs_out = torch.empty((self.n_stats, dim), dtype=torch.float32, device=dev)
        self._tobs_out = torch.zeros((self.n_stats, dim), dtype=torch.float32, device=dev)
        self._rew_out = torch.empty(self.n_stats, **f64)
        if self._world > 1:
            # one packed row per env: obs | terminal obs | reward | terminated | truncated
            self._pack = torch.empty((self.num_envs, 2 * dim + 3), **f64)
            self._gpack = torch.empty((self.n_stats, 2 * dim + 3), **f64)
        self.old_obs = None
        self.old_reward = None
        self._actions = None

    # SB3 attribute names
    @property
    def obs_rms(self):
        return _RMSView(self._obs_mean, self._obs_var, self._obs_count)

    @property
    def ret_rms(self):
        return _RMSView(self._ret_mean, self._ret_var, self._ret_count)

    @property
    def returns(self):
        return self._mine(self._returns).cpu().numpy().copy()

    def _cfg(self):
        return CfgC(int(self.training), int(self.norm_obs), int(self.norm_reward), float(self.clip_obs),
                    float(self.clip_reward), float(self.gamma), float(self.epsilon))

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    # -- device path ---------------------------------------------------------
    def _kernel_reset(self, n, obs, obs_out):
        rt._check(self.L.ur3e_vecnorm_reset(ctypes.byref(self._st), ctypes.byref(self._cfg()), n, self.dim,
                                            ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(obs_out.data_ptr()),
                                            self._stream()))

    def _kernel_step(self, n, obs, rew, term, trunc, tobs):
        rt._check(self.L.ur3e_vecnorm_step(ctypes.byref(self._st), ctypes.byref(self._cfg()), n, self.dim,
                                           *[ctypes.c_void_p(t.data_ptr()) for t in (obs, rew, term, trunc, tobs,
                                                                                    self._obs_out, self._rew_out,
                                                                                    self._tobs_out)],
                                           self._stream()))

    def _gather(self, obs, tobs=None, rew=None, term=None, trunc=None):
        """All ranks' shard outputs in global env-id order (one all-gather of packed rows)."""
        import torch.distributed as dist
        d = self.dim
        p = self._pack
        p[:, :d].copy_(obs)
        if tobs is not None:
            p[:, d:2 * d].copy_(tobs)
            p[:, 2 * d].copy_(rew)
            p[:, 2 * d + 1].copy_(term)
            p[:, 2 * d + 2].copy_(trunc)
        dist.all_gather_into_tensor(self._gpack, p, group=self.group)
        g = self._gpack
        u8 = self.torch.uint8
        return (g[:, :d].contiguous(), g[:, d:2 * d].contiguous(), g[:, 2 * d].contiguous(),
                g[:, 2 * d + 1].to(u8), g[:, 2 * d + 2].to(u8))

    def _mine(self, t):
        lo = self._rank * self.num_envs
        return t[lo:lo + self.num_envs]

    def reset_torch(self):
        obs = self.venv.stepper.reset()
        self.old_obs = obs
        gobs = self._gather(obs)[0] if self._world > 1 else obs
        self._kernel_reset(self.n_stats, gobs, self._obs_out)
        return self._mine(self._obs_out) if self.norm_obs else obs

    def step_torch(self, actions):
        """(normalised obs f32, normalised reward, terminated, truncated, normalised terminal obs f32)
        as device tensors for this rank's envs; raw step outputs stay in old_obs / old_reward."""
        obs, rew, term, trunc, tobs = self.venv.step_torch(actions)
        self.old_obs, self.old_reward = obs, rew
        self._last = (term, trunc, tobs)
        if self._world > 1:
            gobs, gtobs, grew, gterm, gtrunc = self._gather(obs, tobs, rew, term, trunc)
            self._kernel_step(self.n_stats, gobs, grew, gterm, gtrunc, gtobs)
        else:
            self._kernel_step(self.n_stats, obs, rew, term, trunc, tobs)
        o = self._mine(self._obs_out) if self.norm_obs else obs
        to = self._mine(self._tobs_out) if self.norm_obs else tobs
        return o, self._mine(self._rew_out), term, trunc, to

    def normalize_obs_torch(self, obs):
        obs = obs.to(device=self.device, dtype=self.torch.float64).contiguous()
        if not self.norm_obs:
            return obs
        out = self.torch.empty(obs.shape, dtype=self.torch.float32, device=self.device)
        n = obs.numel() // self.dim
        rt._check(self.L.ur3e_vecnorm_normalize_obs(ctypes.byref(self._st), ctypes.byref(self._cfg()), n, self.dim,
                                                    ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                    self._stream()))
        return out

    # -- SB3 VecEnv interface --------------------------------------------------
    def reset(self):
        self.venv._ep_ret[:] = 0
        self.venv._ep_len[:] = 0
        return self.reset_torch().cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        obs, rew, term, trunc, tobs = self.step_torch(self._actions)
        # Monitor's episode return uses the raw reward (Monitor sits inside VecNormalize in SB3)
        _, dones, infos = self.venv.episode_infos(self.old_reward, term, trunc, tobs)
        return obs.cpu().numpy(), rew.cpu().numpy(), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def normalize_obs(self, obs):
        import torch
        return self.normalize_obs_torch(torch.as_tensor(np.asarray(obs, dtype=np.float64))).cpu().numpy()

    def normalize_reward(self, reward):
        reward = np.asarray(reward, dtype=np.float64)
        if self.norm_reward:
            # scalar work on host values already read back; identical expression to SB3
            return np.clip(reward / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward, self.clip_reward)
        return reward

    def get_original_obs(self):
        return self.old_obs.cpu().numpy().copy()

    def get_original_reward(self):
        return self.old_reward.cpu().numpy().copy()

    def close(self):
        self.venv.close()

    def save(self, path):
        """Write the statistics and settings to exactly `path` (train_rl.py:90 names it `...pkl`;
        np.savez on a str would append `.npz`, so it gets an open file instead)."""
        write_stats(path, obs_mean=self.obs_rms.mean, obs_var=self.obs_rms.var, obs_count=self.obs_rms.count,
                    ret_mean=self.ret_rms.mean, ret_var=self.ret_rms.var, ret_count=self.ret_rms.count,
                    cfg=np.array([self.training, self.norm_obs, self.norm_reward, self.clip_obs, self.clip_reward,
                                  self.gamma, self.epsilon], dtype=np.float64))

    @classmethod
    def load(cls, path, venv, group=None):
        """Load statistics written by save() (train_rl.py:49 / evaluate_rl.py:30 pass the path save() got).
        SB3's VecNormalize.load reads a pickle of the whole wrapper; pickles are never loaded here (they
        execute code), so an SB3 file is refused with a clear message instead of failing inside np.load.
        `group`: the process group of a multi-rank run, as in __init__ (the statistics stay global)."""
        z = read_stats(path)
        c = z["cfg"]
        self = cls(venv, training=bool(c[0]), norm_obs=bool(c[1]), norm_reward=bool(c[2]), clip_obs=float(c[3]),
                   clip_reward=float(c[4]), gamma=float(c[5]), epsilon=float(c[6]), group=group)
        t = self.torch
        self._obs_mean.copy_(t.from_numpy(z["obs_mean"]))
        self._obs_var.copy_(t.from_numpy(z["obs_var"]))
        self._obs_count.fill_(float(z["obs_count"]))
        self._ret_mean.fill_(float(z["ret_mean"]))
        self._ret_var.fill_(float(z["ret_var"]))
        self._ret_count.fill_(float(z["ret_count"]))
        return self

    def __getattr__(self, name):
        if name in ("venv",):
            raise AttributeError(name)
        return getattr(self.venv, name)
