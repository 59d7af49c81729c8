"""Batched scripted pick-and-place: controller/move_l_mug.py:16-98 for N envs on one GPU.

Per env, as the reference's main():
  reset_with_mug(m, d, reset_mode, keyframe="down")            gym_utils.py:82-93
  init_r = get_site_xrotvec(tcp); start = get_task_space_state  controller_func.py:191-200
  pick  = [get_mug_xpos (handle_site), init_r, 0.5]
  place = [get_ghost_xpos, init_r, 1]
  traj  = build_traj_l_pick_place(start, [pick, place])        build_traj.py:28-59 (7200 rows)
  for t: u = pid_task_ctrl(traj[t]); mj_step; traj_true[t] = get_task_space_state

The controller and mj_step run inside the step library (task UR3E_TASK_TRAJ_L, one
substep per row); trajectory rows are evaluated on the GPU (PickPlaceTorch).  The
task-space state is computed on the device (ur3e_batch_get_task_space_state): the
stale-kinematics carry (tcp site pose of the last forward), scipy's matrix -> rotvec
conversion restated (utils/utils.py:158-162), and the pad touch sensors compared
lexicographically with (0.1, 0.1) (utils/utils.py:238-245); actuator_frc is the
committed mjData.actuator_force (ur3e_batch_get_actuator_force).

Out of scope: the viewer, CSV/plot logging (controller/aux.py cleanup).
"""
from __future__ import annotations

import numpy as np

from .build_traj import PickPlaceTorch

NOISE = {"deterministic": 0, "high": 1, "med": 2, "low": 3}


def task_space_state(batch, out=None):
    """get_task_space_state for all envs: [N, 7] = tcp xpos, tcp rotvec, boolean grasp contact, computed
    on the device (ur3e_batch_get_task_space_state); `out` may be a row of a recording buffer."""
    if out is None:
        return batch.get_task_space_state()
    batch._chk(batch.L.ur3e_batch_get_task_space_state(batch.h, batch.out_ptr(out, 7, "task_space_state"),
                                                       batch._stream()))
    return out


class MoveLMug:
    """N scripted pick-and-place episodes stepping in lock-step."""

    def __init__(self, n_envs: int, reset_mode: str = "deterministic", device: int = 0, seed: int = 0,
                 envs_per_block: int = 0, sensors: bool = False, config_yaml_path: str | None = None,
                 model: str = "main", tier_con_cap: int = 0):
        """sensors=True also keeps the full mjData.sensordata (incl. the torque sensors) readable through
        batch.get_sensordata() after a step, at the cost of the full-capacity kernel (see
        ur3e_config_t.sensors).  The reference's per-row records -- traj_true (get_task_space_state) and
        actuator_frc (get_jnt_torques), move_l_mug.py:80-81 -- need no sensors flag: run(record=True)
        fills them on the device every row, in every tier.  model="main_mesh" runs main.xml compiled with
        convex meshes (tools/make_main_meshes.py) in the mesh-capable tier set."""
        import torch
        from .. import gains
        from .. import runtime as rt
        self.torch = torch
        md, mc = rt.load_model(model)
        self.md = md
        # controller/move_l_mug.py:20-26: gains from config_l_mug.yml
        cfg = rt.make_config(task=rt.TASK_TRAJ_L, frame_skip=1, max_episode_steps=0, auto_reset=False,
                             reset_noise=NOISE[reset_mode], reset_key=md["id_key_down"], model=md, seed=seed,
                             envs_per_block=envs_per_block, sensors=sensors, tier_con_cap=tier_con_cap,
                             task_gains=gains.task_gains(config_yaml_path))
        self.batch = rt.Batch(mc, cfg, n_envs, device=device)   # reset_with_mug (keyframe + forward)
        obs = self.batch.obs
        start = task_space_state(self.batch)
        init_r = start[:, 3:6]
        n = n_envs
        half = torch.full((n, 1), 0.5, dtype=torch.float64, device=obs.device)
        one = torch.ones((n, 1), dtype=torch.float64, device=obs.device)
        self.pick = torch.cat([obs[:, 3:6], init_r, half], dim=1)
        self.place = torch.cat([obs[:, 6:9], init_r, one], dim=1)
        self.start = start
        self.traj = PickPlaceTorch(start, self.pick, self.place)
        self.T = self.traj.T
        self.t = 0

    def step(self):
        """One trajectory row for all envs: pid_task_ctrl + 1 mj_step."""
        row = self.traj.row(self.t)
        self.batch.step(row)
        self.t += 1
        return row

    def run(self, steps: int | None = None, record: bool = False, record_every: int = 0):
        """Run `steps` rows (default: the rest of the 7200-row trajectory).
        record=True: as the reference's loop (move_l_mug.py:67-81), every row's traj_true
        (get_task_space_state after mj_step) and actuator_frc (get_jnt_torques) go into device buffers
        [steps, N, 7], returned as (traj_true, actuator_frc).  record_every > 0 instead returns
        traj_true samples {t: [N, 7]} every record_every rows."""
        torch = self.torch
        steps = self.T - self.t if steps is None else min(steps, self.T - self.t)
        if record:
            dev = self.batch.device
            traj_true = torch.empty((steps, self.batch.n, 7), dtype=torch.float64, device=dev)
            act_frc = torch.empty((steps, self.batch.n, self.batch.nu), dtype=torch.float64, device=dev)
            for i in range(steps):
                self.step()
                task_space_state(self.batch, traj_true[i])
                self.batch.get_actuator_force(act_frc[i])
            return traj_true, act_frc
        rec = {}
        for _ in range(steps):
            self.step()
            if record_every and self.t % record_every == 0:
                rec[self.t] = task_space_state(self.batch)
        return rec

    def actuator_frc(self):
        """[N, 7] get_jnt_torques (utils/utils.py:201-211): the 7 actuatorfrc sensors in name order
        (= main.xml's actuator order), i.e. mjData.actuator_force of the last forward"""
        return self.batch.get_actuator_force()

    def close(self):
        self.batch.close()


def main(n_envs: int = 4096, steps: int | None = None):  # pragma: no cover - GPU script
    import time
    import torch
    drv = MoveLMug(n_envs)
    t0 = time.perf_counter()
    drv.run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = task_space_state(drv.batch)
    obs = drv.batch.obs
    print(f"{n_envs} envs x {drv.t} rows: {n_envs * drv.t / dt:.0f} env-steps/s; "
          f"mean handle z {obs[:, 5].mean().item():.4f}; grasp flag mean {st[:, 6].mean().item():.3f}")
    drv.close()


if __name__ == "__main__":  # pragma: no cover
    import sys
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096, int(sys.argv[2]) if len(sys.argv) > 2 else None)
