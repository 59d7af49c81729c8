"""Multi-GPU env sharding (one process per GPU, torch.distributed).

SURVEY.md §8(e): envs are independent, so global env ids are split into
contiguous per-rank ranges (rank r owns [r*n_local, (r+1)*n_local)); every
per-env result is invariant to the GPU count because reset noise is keyed by
the global id (the local batch is created with env_id_offset = r*n_local).
The only exchange on the data path is the policy boundary that SB3's
SubprocVecEnv pipes carry in the reference (train_rl.py:38-44): actions are
scattered from the policy rank and (obs, reward, terminated, truncated,
terminal_obs) are gathered to it -- over RCCL (backend "nccl") on MI355X, or
gloo in CPU tests.

Widths come from the local stepper, so every registered id shards: ur3e-v2 /
imitation_indirect (24-d obs, 4-d action), ur3e-v0 (13-d obs, 4-d action) and
imitation_direct (13-d obs, nu-d ctrl action).  Payload per rank per step:
n_local*(2*obs_dim+3) doubles up, n_local*act_dim doubles down (ur3e-v2 at
4096 envs: 1.6 MB / 0.13 MB), latency-bound on one xGMI link.  All send and
receive buffers are allocated once; a step packs into them in place and the
gathered rows are views of one [world, n_local, width] buffer (no torch.cat).
"""
from __future__ import annotations


class ShardedEnvs:
    """Rank-local batch + collective gather/scatter to `root`.

    `local` is any stepper with reset() -> obs [n, obs_dim] and
    step(actions [n, act_dim]) -> (obs, reward, terminated, truncated, terminal_obs)
    returning torch tensors (ur3e_amd.runtime.Batch on a GPU).  obs_dim / act_dim
    default to the stepper's own `obs_dim` / `act_dim` attributes.
    """

    def __init__(self, local, n_local: int, root: int = 0, group=None, obs_dim: int | None = None,
                 act_dim: int | None = None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.local = local
        self.n_local = n_local
        self.root = root
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.num_envs = n_local * self.world
        self.obs_dim = int(obs_dim if obs_dim is not None else local.obs_dim)
        self.act_dim = int(act_dim if act_dim is not None else local.act_dim)
        od = self.obs_dim
        # payload row: obs | reward | terminated | truncated | terminal_obs
        self.width = 2 * od + 3
        dev = self._dev()
        f64 = dict(dtype=torch.float64, device=dev)
        self._send = torch.zeros((n_local, self.width), **f64)
        self._act = torch.empty((n_local, self.act_dim), **f64)
        if self.rank == root:
            self._recv = torch.empty((self.world, n_local, self.width), **f64)
            self._recv_parts = list(self._recv.unbind(0))  # contiguous views, one per rank
        else:
            self._recv, self._recv_parts = None, None

    def _dev(self):
        return self.local.obs.device if hasattr(self.local, "obs") else self.torch.device("cpu")

    def _gather(self):
        self.dist.gather(self._send, self._recv_parts, dst=self.root, group=self.group)
        return None if self._recv is None else self._recv.view(self.num_envs, self.width)

    def _pack(self, obs, rew, term, trunc, tobs):
        od, p = self.obs_dim, self._send
        p[:, :od].copy_(obs)
        p[:, od].copy_(rew)
        p[:, od + 1].copy_(term)
        p[:, od + 2].copy_(trunc)
        p[:, od + 3:].copy_(tobs)

    def _unpack(self, g):
        od = self.obs_dim
        return g[:, :od], g[:, od], g[:, od + 1] > 0.5, g[:, od + 2] > 0.5, g[:, od + 3:]

    def reset(self):
        """Reset every shard; root receives the [num_envs, obs_dim] initial observations."""
        obs = self.local.reset()
        self._send.zero_()
        self._send[:, :self.obs_dim].copy_(obs)
        g = self._gather()
        return None if g is None else g[:, :self.obs_dim].clone()

    def step(self, actions_global=None):
        """Root passes actions for all envs [num_envs, act_dim]; other ranks pass None.
        Returns the gathered (obs, reward, terminated, truncated, terminal_obs) on root, None elsewhere.
        The returned tensors are views of the receive buffer, valid until the next step."""
        t = self.torch
        if self.rank == self.root:
            a = actions_global.to(self._act.device, t.float64).reshape(self.world, self.n_local, self.act_dim)
            chunks = list(a.contiguous().unbind(0))
            self.dist.scatter(self._act, chunks, src=self.root, group=self.group)
        else:
            self.dist.scatter(self._act, None, src=self.root, group=self.group)
        self._pack(*self.local.step(self._act))
        g = self._gather()
        return None if g is None else self._unpack(g)
