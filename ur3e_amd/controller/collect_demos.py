"""Batched expert-demonstration collection: gymnasium_src/scripts/imitation_rl/collect_demos.py:86-189
for N demos at once on one GPU.

Per demo, as the reference's collect_expert_demonstrations():
  reset_with_mug(m, d, reset_mode, keyframe="down", noise_mag)           gym_utils.py:82-93
  init_r = get_site_xrotvec(tcp); place = [ghost xpos, init_r, 1]; pick = [mug xpos, init_r, 0.0]
  traj = build_traj_l_pick_place_imitation_augmented(get_task_space_state, [pick, place], hold)
  obs = [get_obs]
  for t in range(T):  u = pid_task_ctrl(traj[t]); d.ctrl = u; mj_step
      if t % down_sample == 0: acts += [traj[t, :3] + u[-1]] (indirect) or [u] (direct); obs += [get_obs]
  Trajectory(obs, acts, infos=[{}...], terminal=True)

Here the N demos step in lock-step inside the step library (task UR3E_TASK_TRAJ_L, one mj_step per
row); the augmented trajectories are built on the GPU (AugmentedPickPlaceTorch, 10500 rows each,
time-major in HBM); observations and actions are recorded into device tensors and copied to the host
once at the end.  get_obs (collect_demos.py:60-83) is the ur3e-v2 observation, emitted by the
library for the scripted task.  u is read back with ur3e_batch_get_ctrl (d.ctrl after the step).

Noise: the reference draws reset and trajectory noise from the unseeded global np.random; here the
reset noise is the library's Philox stream (keyed by seed and demo id) and the trajectory noise is
torch.rand on the device (seeded), or any [N, 7500, 7] uniform tensor passed as `noise`.

Out of scope: the viewer and the `imitation` package's training loops.
"""
from __future__ import annotations

import dataclasses
import os
import pickle

import numpy as np

from .build_traj import AUG_NOISE_ROWS, AugmentedPickPlaceTorch
from .move_l_mug import NOISE, task_space_state


@dataclasses.dataclass(frozen=True)
class Trajectory:
    """Field-compatible stand-in for imitation.data.types.Trajectory (not installed here)."""
    obs: np.ndarray
    acts: np.ndarray
    infos: np.ndarray | None
    terminal: bool

    def __len__(self):
        return len(self.acts)


def _trajectory_cls():
    try:  # pragma: no cover - the imitation package is not in this image
        from imitation.data.types import Trajectory as T
        return T
    except Exception:
        return Trajectory


class DemoCollector:
    """N expert demos (collect_demos.py settings: action_mode, reset_mode, noise_mag, down_sample)."""

    def __init__(self, n_demos: int, action_mode: str = "indirect", reset_mode: str = "stochastic",
                 noise_mag: str = "low", down_sample: int = 1, seed: int = 0, device: int = 0, noise=None,
                 envs_per_block: int = 0, config_yaml_path: str | None = None):
        import torch
        from .. import gains
        from .. import runtime as rt
        if action_mode not in ("indirect", "direct"):
            raise ValueError(f"action_mode must be 'indirect' or 'direct', got {action_mode!r}")
        if reset_mode not in ("stochastic", "deterministic"):
            raise ValueError(f"reset_mode must be 'stochastic' or 'deterministic', got {reset_mode!r}")
        self.torch = torch
        self.action_mode = action_mode
        self.down_sample = int(down_sample)
        md, mc = rt.load_model("main")
        rn = NOISE[noise_mag] if reset_mode == "stochastic" else 0
        cfg = rt.make_config(task=rt.TASK_TRAJ_L, frame_skip=1, max_episode_steps=0, auto_reset=False,
                             reset_noise=rn, reset_key=md["id_key_down"], model=md, seed=seed,
                             envs_per_block=envs_per_block,
                             task_gains=gains.task_gains(config_yaml_path))  # collect_demos.py:89-94
        self.batch = rt.Batch(mc, cfg, n_demos, device=device)
        dev = self.batch.device
        n = n_demos
        obs0 = self.batch.obs.clone()
        start = task_space_state(self.batch)
        init_r = start[:, 3:6]
        zero = torch.zeros((n, 1), dtype=torch.float64, device=dev)
        one = torch.ones((n, 1), dtype=torch.float64, device=dev)
        self.place = torch.cat([obs0[:, 6:9], init_r, one], dim=1)
        self.pick = torch.cat([obs0[:, 3:6], init_r, zero], dim=1)
        self.start = start
        if noise is None:
            g = torch.Generator(device=dev)
            g.manual_seed(int(seed) + 0x5EED)
            noise = torch.rand((n, AUG_NOISE_ROWS, 7), dtype=torch.float64, device=dev, generator=g)
        self.traj = AugmentedPickPlaceTorch(start, self.pick, self.place, noise.to(dev))
        del noise
        self.T = self.traj.T
        self.n = n
        self.obs0 = obs0
        self.t = 0

    def run(self, steps: int | None = None):
        """Step `steps` rows (default: the whole trajectory). Returns device tensors
        obs [K+1, N, 24] and acts [K, N, adim] (time-major), K = ceil(steps / down_sample)."""
        torch = self.torch
        steps = self.T if steps is None else min(int(steps), self.T)
        ds = self.down_sample
        k = (steps + ds - 1) // ds
        adim = 4 if self.action_mode == "indirect" else self.batch.nu
        dev = self.batch.device
        obs = torch.empty((k + 1, self.n, self.batch.obs_dim), dtype=torch.float64, device=dev)
        acts = torch.empty((k, self.n, adim), dtype=torch.float64, device=dev)
        obs[0] = self.obs0
        j = 0
        for t in range(steps):
            row = self.traj.row(t)
            self.batch.step(row)
            if t % ds == 0:
                u = self.batch.get_ctrl()
                if self.action_mode == "indirect":
                    acts[j, :, :3] = row[:, :3]
                    acts[j, :, 3] = u[:, -1]
                else:
                    acts[j] = u
                obs[j + 1] = self.batch.obs
                j += 1
        self.t = steps
        return obs, acts

    def trajectories(self, obs, acts):
        """Per-demo Trajectory objects (host numpy), as collect_demos.py:176-181."""
        T = _trajectory_cls()
        o = obs.transpose(0, 1).cpu().numpy()
        a = acts.transpose(0, 1).cpu().numpy()
        infos = np.array([{} for _ in range(a.shape[1])])
        return [T(obs=o[i], acts=a[i], infos=infos.copy(), terminal=True) for i in range(self.n)]

    def close(self):
        self.batch.close()


def stack_expert_trajectories(trajectories, history_len):
    """collect_demos.py:21-57: frame-stack each trajectory's obs with a history of `history_len`,
    padding the start by repeating the first frame.  Vectorised: obs[i] -> obs[max(0, i-h+1) .. i]."""
    out = []
    for traj in trajectories:
        o = np.asarray(traj.obs)
        idx = np.arange(len(o))[:, None] + np.arange(-history_len + 1, 1)[None, :]
        stacked = o[np.clip(idx, 0, None)]
        out.append(type(traj)(obs=stacked, acts=traj.acts, infos=traj.infos, terminal=traj.terminal))
    return out


def save_demos(trajectories, save_path, resume_collecting=False):
    """collect_demos.py:192-211: append to a pickle of trajectories (this code's own files only)."""
    d = os.path.dirname(save_path)
    if d:
        os.makedirs(d, exist_ok=True)
    existing = []
    if resume_collecting and os.path.exists(save_path):
        with open(save_path, "rb") as f:
            existing = pickle.load(f)
    existing.extend(trajectories)
    with open(save_path, "wb") as f:
        pickle.dump(existing, f)
    return len(existing)


def main(n_demos: int = 4096, action_mode: str = "indirect"):  # pragma: no cover - GPU script
    import time
    import torch
    col = DemoCollector(n_demos, action_mode=action_mode)
    t0 = time.perf_counter()
    obs, acts = col.run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{n_demos} demos x {col.T} rows in {dt:.2f} s: {n_demos / dt:.1f} demos/s, "
          f"{n_demos * col.T / dt:.0f} env-steps/s; final mug z mean {obs[-1, :, 5].mean().item():.4f}")
    col.close()


if __name__ == "__main__":  # pragma: no cover
    import sys
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096, sys.argv[2] if len(sys.argv) > 2 else "indirect")
