"""Device-resident PPO driving the batched env (BASELINE config C5).

Replaces `stable_baselines3.PPO("MlpPolicy", VecNormalize(venv), ...)` as configured in
gymnasium_src/scripts/regular_rl/rl/train_rl.py:60-73 with gymnasium_src/config/config_rl.yml
(net_arch [256, 256], lr 3e-4, batch 256, n_epochs 30, gamma 0.99, gae_lambda 0.95, ent_coef 0.01;
SB3 defaults for the rest: clip_range 0.2, vf_coef 0.5, max_grad_norm 0.5, Adam eps 1e-5,
normalize_advantage, state-independent log_std initialised to 0, tanh MLPs with orthogonal init).
No feature extractor: train_rl.py:123 reads `hyperparameters.get("feature_encoder")` while the
yml key is `feature_extractor`, so the reference's transformer / frame-stack branch (:26-35) is
never taken and the policy is the plain MLP above.  SB3 itself is not installed in this image; the algorithm follows stable_baselines3==2.x
(`PPO.train`, `OnPolicyAlgorithm.collect_rollouts`, `RolloutBuffer.compute_returns_and_advantage`).

MI355X layout: the env, the on-device VecNormalize, the rollout buffer and the policy all live on
one GPU and share torch's current stream, so a rollout step is env kernel -> normalisation kernel ->
policy forward with no host round trip.  With several ranks (one process per GPU) each rank steps its
own env shard and keeps a policy replica; gradients are flattened into ONE buffer and all-reduced
(averaged) per minibatch, a single RCCL call over xGMI instead of one per parameter tensor.

The env object only needs `num_envs`, `action_space` (low/high), `reset_torch()` and
`step_torch(actions) -> (obs f32, reward, terminated, truncated, terminal_obs f32)`: the GPU
`VecNormalize` provides it, and tests use a CPU stand-in with the same interface.
"""
from __future__ import annotations

import math
import time

import torch
import torch.nn as nn


def _mlp(sizes, gain):
    layers = []
    for i in range(len(sizes) - 1):
        lin = nn.Linear(sizes[i], sizes[i + 1])
        nn.init.orthogonal_(lin.weight, gain=gain)
        nn.init.zeros_(lin.bias)
        layers += [lin, nn.Tanh()]
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    """SB3 ActorCriticPolicy for a Box action space with net_arch=[256, 256]: separate pi / vf MLPs
    over the flattened observation, Gaussian head with a state-independent log_std."""

    def __init__(self, obs_dim: int, act_dim: int, net_arch=(256, 256), log_std_init: float = 0.0):
        super().__init__()
        self.pi_net = _mlp([obs_dim, *net_arch], gain=math.sqrt(2))
        self.vf_net = _mlp([obs_dim, *net_arch], gain=math.sqrt(2))
        self.action_net = nn.Linear(net_arch[-1], act_dim)
        self.value_net = nn.Linear(net_arch[-1], 1)
        nn.init.orthogonal_(self.action_net.weight, gain=0.01)
        nn.init.zeros_(self.action_net.bias)
        nn.init.orthogonal_(self.value_net.weight, gain=1.0)
        nn.init.zeros_(self.value_net.bias)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))

    def dist(self, obs):
        mean = self.action_net(self.pi_net(obs))
        # validate_args=False: the argument checks synchronise with the host every rollout step
        return torch.distributions.Normal(mean, self.log_std.exp().expand_as(mean), validate_args=False)

    def value(self, obs):
        return self.value_net(self.vf_net(obs)).squeeze(-1)

    def evaluate(self, obs, actions):
        d = self.dist(obs)
        return self.value(obs), d.log_prob(actions).sum(-1), d.entropy().sum(-1)


def compute_gae(rewards, values, episode_starts, last_values, dones, gamma, lam):
    """RolloutBuffer.compute_returns_and_advantage: rewards/values/episode_starts [T, N];
    `dones` are the done flags after the last step. Returns (advantages, returns)."""
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    last = torch.zeros_like(last_values)
    for t in reversed(range(T)):
        if t == T - 1:
            nonterm = 1.0 - dones.to(rewards.dtype)
            nv = last_values
        else:
            nonterm = 1.0 - episode_starts[t + 1]
            nv = values[t + 1]
        delta = rewards[t] + gamma * nv * nonterm - values[t]
        last = delta + gamma * lam * nonterm * last
        adv[t] = last
    return adv, adv + values


class PPO:
    def __init__(self, env, n_steps: int = 16, batch_size: int = 256, n_epochs: int = 30, learning_rate: float = 3e-4,
                 gamma: float = 0.99, gae_lambda: float = 0.95, clip_range: float = 0.2, ent_coef: float = 0.01,
                 vf_coef: float = 0.5, max_grad_norm: float = 0.5, net_arch=(256, 256), device=None, seed: int = 0,
                 group=None, graphs=None):
        self.env = env
        self.n_envs = env.num_envs
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        low = torch.as_tensor(env.action_space.low, dtype=torch.float32, device=self.device)
        high = torch.as_tensor(env.action_space.high, dtype=torch.float32, device=self.device)
        self.low, self.high = low, high
        self.obs_dim = env.observation_space.shape[0]
        self.act_dim = low.numel()
        self.n_steps, self.batch_size, self.n_epochs = n_steps, batch_size, n_epochs
        self.gamma, self.lam, self.clip, self.ent_coef, self.vf_coef = gamma, gae_lambda, clip_range, ent_coef, vf_coef
        self.max_grad_norm = max_grad_norm
        self.group = group
        torch.manual_seed(seed)
        self.policy = ActorCritic(self.obs_dim, self.act_dim, net_arch).to(self.device)
        if group is not None:  # identical replicas: broadcast rank 0's initial weights
            import torch.distributed as dist
            for p in self.policy.parameters():
                dist.broadcast(p.data, src=0, group=group)
        # gradients live in ONE flat buffer (each parameter's .grad is a view of it): the multi-rank
        # average is a single all-reduce on that buffer, with no flatten / unflatten copies
        params = list(self.policy.parameters())
        self._flat_grad = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=self.device)
        off = 0
        for p in params:
            p.grad = self._flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        # on the GPU the minibatch update is replayed from HIP graphs (a batch-256 update is a few
        # hundred tiny kernels, launch-bound when issued one by one); Adam keeps its step count on
        # the device for that (capturable)
        self.use_graphs = (self.device.type == "cuda") if graphs is None else bool(graphs)
        self.opt = torch.optim.Adam(params, lr=learning_rate, eps=1e-5, capturable=self.use_graphs)
        self._graphs = None
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        T, N, f = n_steps, self.n_envs, dict(dtype=torch.float32, device=self.device)
        self.buf_obs = torch.zeros((T, N, self.obs_dim), **f)
        self.buf_act = torch.zeros((T, N, self.act_dim), **f)
        self.buf_rew = torch.zeros((T, N), **f)
        self.buf_start = torch.zeros((T, N), **f)
        self.buf_val = torch.zeros((T, N), **f)
        self.buf_logp = torch.zeros((T, N), **f)
        self._noise = torch.zeros((T, N, self.act_dim), **f)
        self._obs = None
        self._start = torch.ones(N, **f)
        self.num_timesteps = 0
        self.stats = {}

    # -- rollout ---------------------------------------------------------------
    def _rollout_step(self, t: int):
        """One env step at rollout index t (persistent tensors; no host synchronisation).
        Launch count is what limits a 4,096-env rollout step, so: the sampling noise and the
        log-probabilities are handled for the whole rollout at once (log_std is constant during a
        rollout: log N(mean + std*eps) = -eps^2/2 - log_std - log(2 pi)/2), and the value of the next
        observation and of the terminal observation share one critic pass over 2N rows."""
        N = self.n_envs
        obs = self._obs
        act = self.policy.action_net(self.policy.pi_net(obs)) + self._std * self._noise[t]
        clipped = torch.maximum(torch.minimum(act, self.high), self.low)
        nobs, rew, term, trunc, tobs = self.env.step_torch(clipped.to(torch.float64))
        self._vin[:N].copy_(nobs)
        self._vin[N:].copy_(tobs)
        v2 = self.policy.value(self._vin)
        term, trunc = term.bool(), trunc.bool()
        # SB3 timeout bootstrap: truncated-not-terminated envs get gamma * V(terminal obs); evaluated
        # for every env and masked, so the rollout never waits on the host for an any()
        rew = rew.to(torch.float32) + self.gamma * torch.where(trunc & ~term, v2[N:], torch.zeros_like(v2[N:]))
        self.buf_obs[t].copy_(obs)
        self.buf_act[t].copy_(act)
        self.buf_rew[t].copy_(rew)
        self.buf_start[t].copy_(self._start)
        self.buf_val[t].copy_(self._val)
        self._val.copy_(v2[:N])
        self._obs.copy_(nobs)  # the env reuses its output buffers: copy, never alias
        self._start.copy_((term | trunc).to(torch.float32))

    @torch.no_grad()
    def collect_rollouts(self):
        if self._obs is None:
            self._obs = self.env.reset_torch().to(torch.float32).clone()
            self._val = self.policy.value(self._obs)
            self._vin = torch.empty((2 * self.n_envs, self.obs_dim), dtype=torch.float32, device=self.device)
        else:  # the critic changed in train(): value the carried-over observation with the new one
            self._val = self.policy.value(self._obs)
        # all sampling noise of the rollout in one draw
        self._noise.normal_(generator=self.gen)
        self._std = self.policy.log_std.exp()
        for t in range(self.n_steps):
            self._rollout_step(t)
        ls = self.policy.log_std
        self.buf_logp.copy_(-0.5 * self._noise.pow(2).sum(-1) - (ls.sum() + 0.5 * math.log(2 * math.pi) * ls.numel()))
        last_val = self._val
        self.adv, self.ret = compute_gae(self.buf_rew, self.buf_val, self.buf_start, last_val, self._start > 0,
                                         self.gamma, self.lam)
        self.num_timesteps += self.n_steps * self.n_envs

    # -- update ----------------------------------------------------------------
    def _allreduce_grads(self):
        import torch.distributed as dist
        dist.all_reduce(self._flat_grad, group=self.group)
        self._flat_grad /= dist.get_world_size(self.group)

    def _loss(self, idx):
        """SB3 PPO.train minibatch loss (clipped surrogate, value MSE, entropy bonus)."""
        v, logp, ent = self.policy.evaluate(self._obs_all[idx], self._act_all[idx])
        adv = self._adv_s[idx]
        if adv.numel() > 1:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        ratio = torch.exp(logp - self._logp_all[idx])
        pg = -torch.min(adv * ratio, adv * ratio.clamp(1 - self.clip, 1 + self.clip)).mean()
        vf = torch.nn.functional.mse_loss(self._ret_s[idx], v)
        ent_loss = -ent.mean()
        return pg + self.ent_coef * ent_loss + self.vf_coef * vf, pg, vf, ent_loss

    def _backward(self, idx):
        self._flat_grad.zero_()
        loss, pg, vf, ent_loss = self._loss(idx)
        loss.backward()
        return pg.detach(), vf.detach(), ent_loss.detach()

    def _apply(self):
        nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
        self.opt.step()

    def _minibatch_eager(self, idx):
        out = self._backward(idx)
        if self.group is not None:
            self._allreduce_grads()
        self._apply()
        return out

    def _capture(self):
        """Two graphs per minibatch: (zero grads, forward, backward) and (clip, Adam step); the
        multi-rank gradient average runs between them as one eager RCCL all-reduce."""
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga):
            self._g_out = self._backward(self._g_idx)
        with torch.cuda.graph(gb, pool=ga.pool()):
            self._apply()
        self._graphs = (ga, gb)

    def _minibatch_graph(self, idx):
        self._g_idx.copy_(idx)
        self._graphs[0].replay()
        if self.group is not None:
            self._allreduce_grads()
        self._graphs[1].replay()
        return self._g_out

    def train(self):
        T, N = self.n_steps, self.n_envs
        B = self.batch_size
        total = T * N
        self._obs_all = self.buf_obs.reshape(total, -1)
        self._act_all = self.buf_act.reshape(total, -1)
        self._logp_all = self.buf_logp.reshape(-1)
        if getattr(self, "_adv_s", None) is None:  # persistent: the graphs read these addresses
            self._adv_s = torch.empty(total, dtype=torch.float32, device=self.device)
            self._ret_s = torch.empty(total, dtype=torch.float32, device=self.device)
            self._g_idx = torch.zeros(B, dtype=torch.long, device=self.device)
        self._adv_s.copy_(self.adv.reshape(-1))
        self._ret_s.copy_(self.ret.reshape(-1))
        last = None
        warm = 0
        for _ in range(self.n_epochs):
            perm = torch.randperm(total, generator=self.gen, device=self.device)
            for s in range(0, total, B):
                idx = perm[s:s + B]
                if not self.use_graphs or idx.numel() != B:
                    last = self._minibatch_eager(idx)
                elif self._graphs is None and warm < 3:
                    # warm-up before capture (torch.cuda.graphs): real minibatch updates, run on a
                    # side stream so that autograd and the BLAS handles settle outside the capture
                    side = torch.cuda.Stream(device=self.device)
                    side.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(side):
                        last = self._minibatch_eager(idx)
                    torch.cuda.current_stream(self.device).wait_stream(side)
                    warm += 1
                else:
                    if self._graphs is None:
                        self._capture()
                    last = self._minibatch_graph(idx)
        if last is not None:
            self.stats = dict(zip(("policy_gradient_loss", "value_loss", "entropy_loss"), (float(x) for x in last)))

    def learn(self, iterations: int = 1):
        """Returns per-iteration wall times {rollout_s, train_s}."""
        times = []
        for _ in range(iterations):
            t0 = time.perf_counter()
            self.collect_rollouts()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            t1 = time.perf_counter()
            self.train()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            times.append({"rollout_s": t1 - t0, "train_s": time.perf_counter() - t1})
        return times
