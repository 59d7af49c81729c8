"""Test helpers: an oracle-backed CPU stepper with the runtime.Batch interface
(torch CPU tensors), used to test host logic (VecEnv, sharding) without a GPU.
Test infrastructure only."""
import numpy as np


def oracle_config(po, c):
    return po.config_from(c)


class OracleStepper:
    def __init__(self, n, seed=0, env_id_offset=0, max_episode_steps=2500, model="main",
                 env_id="gymnasium_env/ur3e-v2"):
        import torch
        from oracle import pyoracle as po
        from ur3e_amd import runtime as rt
        self.torch = torch
        from ur3e_amd.envs.specs import spec
        s = spec(env_id)
        md, mc = rt.load_model(model)
        cfg = rt.make_config(task=s["task"], frame_skip=s["frame_skip"], max_episode_steps=max_episode_steps,
                             model=md, seed=seed, env_id_offset=env_id_offset, task_gains=s["gains"])
        self.cfg = cfg
        self.ob = po.OracleBatch(mc, oracle_config(po, cfg), n)
        self.n = n
        self.obs = torch.from_numpy(self.ob.obs.copy())
        self.obs_dim = s["obs_dim"]
        self.act_dim = len(s["low"])

    def reset(self):
        return self.torch.from_numpy(self.ob.obs.copy())

    def step(self, actions):
        a = actions.detach().cpu().numpy() if hasattr(actions, "detach") else np.asarray(actions)
        obs, rew, term, trunc, tobs = self.ob.step(a)
        t = self.torch
        return (t.from_numpy(obs), t.from_numpy(rew), t.from_numpy(term), t.from_numpy(trunc), t.from_numpy(tobs))

    def close(self):
        pass


def oracle_pick_place_rows(md, mc, ob):
    """Per-env build_traj_l_pick_place rows [n, 7200, 7] for an OracleBatch created with the
    move_l_mug configuration (controller/move_l_mug.py:36-38: start = tcp pose, pick = handle_site,
    place = ghost, rotation held at the start's rotvec), from the oracle's reset state."""
    from scipy.spatial.transform import Rotation as R
    from oracle import pyoracle as po
    from ur3e_amd.controller.build_traj import build_traj_l_pick_place
    qp = ob.get_state()[0]
    tcp, h = md["id_site_tcp"], md["id_site_handle"]
    rows = []
    for i in range(ob.n):
        fs = po.forward_state(mc, qp[i])
        rv = R.from_matrix(fs["site_xmat"][tcp].reshape(3, 3)).as_rotvec()
        start = np.r_[fs["site_xpos"][tcp], rv, 0.0]
        pick = np.r_[fs["site_xpos"][h], rv, 0.5]
        place = np.r_[ob.obs[i, 6:9], rv, 1.0]
        rows.append(build_traj_l_pick_place(start, [pick, place]))
    return np.stack(rows)
