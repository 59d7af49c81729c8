"""CPU restatement of SB3's VecNormalize statistics and normalisation (numpy).

TEST INFRASTRUCTURE ONLY -- the checker for ur3e_amd/csrc/ur3e_vecnorm.hip; the product package
never imports it.

Restates the third-party stable_baselines3==2.7.0 (reference requirements.txt:100; not vendored in
the reference and not installed here) as used by gymnasium_src/scripts/regular_rl/rl/train_rl.py:57:
  common/running_mean_std.py  RunningMeanStd(epsilon=1e-4): update(arr) -> np.mean/np.var over
                              axis 0 + update_from_moments
  vec_env/vec_normalize.py    VecNormalize.reset / step_wait / normalize_obs (clip, float32) /
                              normalize_reward / _update_reward (returns = returns * gamma + r)
The numpy calls are the ones SB3 makes, so this file's results are SB3's bit-for-bit on the same
inputs; the GPU kernels reproduce numpy's reduction order.
"""
from __future__ import annotations

import numpy as np


class RunningMeanStd:
    def __init__(self, epsilon: float = 1e-4, shape=()):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon

    def update(self, arr):
        batch_mean = np.mean(arr, axis=0)
        batch_var = np.var(arr, axis=0)
        batch_count = arr.shape[0]
        self.update_from_moments(batch_mean, batch_var, batch_count)

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        delta = batch_mean - self.mean
        tot_count = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        m_2 = m_a + m_b + np.square(delta) * self.count * batch_count / (self.count + batch_count)
        new_var = m_2 / (self.count + batch_count)
        new_count = batch_count + self.count
        self.mean, self.var, self.count = new_mean, new_var, new_count


class VecNormalizeRef:
    def __init__(self, num_envs, obs_dim, training=True, norm_obs=True, norm_reward=True, clip_obs=10.0,
                 clip_reward=10.0, gamma=0.99, epsilon=1e-8):
        self.obs_rms = RunningMeanStd(shape=(obs_dim,))
        self.ret_rms = RunningMeanStd(shape=())
        self.clip_obs, self.clip_reward = clip_obs, clip_reward
        self.returns = np.zeros(num_envs)
        self.gamma, self.epsilon = gamma, epsilon
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward

    def normalize_obs(self, obs):
        if self.norm_obs:
            return np.clip((obs - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon),
                           -self.clip_obs, self.clip_obs).astype(np.float32)
        return obs

    def normalize_reward(self, reward):
        if self.norm_reward:
            return np.clip(reward / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward, self.clip_reward)
        return reward

    def reset(self, obs):
        self.returns = np.zeros(len(obs))
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        return self.normalize_obs(obs)

    def step(self, obs, rewards, dones, terminal_obs):
        """step_wait on the wrapped env's outputs; terminal_obs rows of done envs are normalised."""
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        out = self.normalize_obs(obs)
        if self.training:
            self.returns = self.returns * self.gamma + rewards
            self.ret_rms.update(self.returns)
        rew = self.normalize_reward(rewards)
        tobs = {int(i): self.normalize_obs(terminal_obs[i]) for i in np.flatnonzero(dones)}
        self.returns[dones] = 0
        return out, rew, tobs
