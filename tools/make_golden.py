"""Generate golden vectors from the REFERENCE Python (container-only).

Imports the reference (`/root/reference`) with stub `mujoco`/`gymnasium`
modules and records inputs/outputs of the controller,
rotation, trajectory, reward and task-predicate functions on seeded synthetic
inputs.  MuJoCo-dependent inputs (site poses, Jacobians, qfrc_bias, contacts)
are passed in as arrays through fake model/data objects.

Output: tests/golden/reference_golden.npz (+ JSON meta).  Only data leaves this
script; nothing from the reference travels to the GPU box.
"""
import contextlib
import io
import json
import os
import sys
import types

import numpy as np

REF = os.environ.get("UR3E_REFERENCE", "/root/reference")
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
from ur3e_amd.model.compiler import load_json  # noqa: E402


# --------------------------------------------------------------------------- stubs
class _Stub(types.ModuleType):
    def __getattr__(self, n):
        if n.startswith("__"):
            raise AttributeError(n)
        return type(n, (), {})


mj = _Stub("mujoco")


class _mjtObj:
    mjOBJ_BODY = 1
    mjOBJ_JOINT = 3
    mjOBJ_GEOM = 5
    mjOBJ_SITE = 6


mj.mjtObj = _mjtObj
mj.mj_name2id = lambda m, t, name: m._names[t][name]
mj.mj_id2name = lambda m, t, i: {v: k for k, v in m._names[t].items()}[i]


def _jac_site(m, d, jacp, jacr, sid):
    if jacp is not None:
        jacp[:] = d._jacp
    if jacr is not None:
        jacr[:] = d._jacr


mj.mj_jacSite = _jac_site
sys.modules["mujoco"] = mj
sys.modules["mujoco.viewer"] = _Stub("mujoco.viewer")
for n in ["gymnasium", "gymnasium.envs", "gymnasium.envs.registration", "gymnasium.wrappers", "gymnasium.spaces"]:
    sys.modules[n] = _Stub(n)
gm = _Stub("gymnasium.envs.mujoco")
gm.MujocoEnv = type("MujocoEnv", (), {})
sys.modules["gymnasium.envs.mujoco"] = gm
sys.modules["gymnasium"].spaces = sys.modules["gymnasium.spaces"]

sys.path.insert(0, REF)
_cwd = os.getcwd()
os.chdir(REF)
import utils.utils as uu  # noqa: E402

uu.get_joint_torques = uu.get_jnt_torques  # alias shim for the broken import
import controller.controller_func as cf  # noqa: E402
import controller.build_traj as bt  # noqa: E402
import controller.move_j as mvj  # noqa: E402
import controller.move_l as mvl  # noqa: E402
import utils.gym_utils as gu  # noqa: E402
from gymnasium_env.envs.ur3e_env2 import UR3eEnv2  # noqa: E402
from gymnasium_env.envs.ur3e_env import UR3eEnv  # noqa: E402
import yaml  # noqa: E402

with open("controller/config/config_l_mug.yml") as f:
    YML_MUG = yaml.safe_load(f)
with open("controller/config/config_j.yml") as f:
    YML_J = yaml.safe_load(f)
with open("controller/config/config_l.yml") as f:
    YML_L = yaml.safe_load(f)
os.chdir(_cwd)


# --------------------------------------------------------------------------- fakes
class _Obj:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class FakeModel:
    def __init__(self, md):
        self._md = md
        self._names = {
            _mjtObj.mjOBJ_BODY: {n: i for i, n in enumerate(md["body_names"])},
            _mjtObj.mjOBJ_SITE: {n: i for i, n in enumerate(md["site_names"])},
            _mjtObj.mjOBJ_JOINT: {n: i for i, n in enumerate(md["joint_names"])},
            _mjtObj.mjOBJ_GEOM: {n: i for i, n in enumerate(md["geom_names"]) if n},
        }
        self.nv = md["nv"]
        self.nq = md["nq"]
        self.nbody = md["nbody"]
        self.opt = _Obj(timestep=md["timestep"])
        self.actuator_ctrlrange = np.array(md["act_ctrlrange"])
        self.jnt_range = np.array(md["jnt_range"])
        self.body_parentid = np.array(md["body_parentid"])
        self.geom_bodyid = np.array(md["geom_bodyid"])
        self.geom_size = np.array(md["geom_size"])
        self._keys = {n: (np.array(md["key_qpos"][i]), np.array(md["key_qvel"][i]))
                      for i, n in enumerate(md["key_names"])}

    def keyframe(self, name):
        q, v = self._keys[name]
        return _Obj(qpos=q.copy(), qvel=v.copy())


class FakeData:
    def __init__(self, nsite, nbody, nv, nq):
        self.site_xpos = np.zeros((nsite, 3))
        self.site_xmat = np.zeros((nsite, 9))
        self.body_xpos = np.zeros((nbody, 3))
        self.qvel = np.zeros(nv)
        self.qpos = np.zeros(nq)
        self.qfrc_bias = np.zeros(nv)
        self._jacp = np.zeros((3, nv))
        self._jacr = np.zeros((3, nv))
        self.contact = []
        self.ncon = 0

    def site(self, i):
        return _Obj(xpos=self.site_xpos[i], xmat=self.site_xmat[i])

    def body(self, i):
        return _Obj(xpos=self.body_xpos[i])


def rand_rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def main():
    md = load_json(os.path.join(REPO, "ur3e_amd", "assets", "main.model.json"))
    fm = FakeModel(md)
    rng = np.random.default_rng(12345)
    tcp = md["site_names"].index("tcp")
    out = {}

    # ---- A. rotation error (controller_func.get_rot_err, scipy Rotation)
    N = 300
    xm, tg, er = [], [], []
    for k in range(N):
        R = rand_rot(rng)
        if k % 10 == 0:  # near the controller's operating point
            R = np.array(
                [[0, 0, -1], [0, 1, 0], [1, 0, 0]], float) @ rand_rot(rng) if k % 20 == 0 else R
        t = rng.normal(size=3) * (0.1 if k % 3 == 0 else 1.5)
        if k % 7 == 0:
            t = np.array([-1.209, -1.209, 1.209])
        d = FakeData(md["nsite"], md["nbody"], md["nv"], md["nq"])
        d.site_xmat[tcp] = R.reshape(9)
        errs = np.zeros((1, 3))
        e = cf.get_rot_err(0, fm, d, t, errs)
        xm.append(R.reshape(9)); tg.append(t); er.append(e)
    out["rot_xmat"], out["rot_target"], out["rot_err"] = np.array(xm), np.array(tg), np.array(er)

    # ---- B. pid_task_ctrl with config_l_mug gains
    pos_gains = {k: np.diag(v) for k, v in YML_MUG["pos"].items()}
    rot_gains = {k: np.diag(v) for k, v in YML_MUG["rot"].items()}
    N = 200
    ins = dict(traj=[], xpos=[], xmat=[], jac=[], qvel=[], bias=[], ctrl=[])
    for k in range(N):
        d = FakeData(md["nsite"], md["nbody"], md["nv"], md["nq"])
        traj = np.concatenate([rng.uniform([0.05, -0.12, 0], [0.55, 0.38, 0.5]), [-1.209, -1.209, 1.209],
                               [rng.uniform(0, 1)]])
        if k % 4 == 0:
            traj[3:6] = rng.normal(size=3)
        d.site_xpos[tcp] = rng.uniform([0.1, -0.2, 0.05], [0.5, 0.4, 0.4])
        d.site_xmat[tcp] = rand_rot(rng).reshape(9)
        d._jacp = rng.normal(size=(3, md["nv"])) * 0.3
        d._jacr = rng.normal(size=(3, md["nv"]))
        d.qvel = rng.normal(size=md["nv"])
        d.qfrc_bias = rng.normal(size=md["nv"]) * 5
        u = cf.pid_task_ctrl(0, fm, d, traj, pos_gains, rot_gains, np.zeros((1, 3)), np.zeros((1, 3)),
                             np.zeros(3), np.zeros(3))
        ins["traj"].append(traj); ins["xpos"].append(d.site_xpos[tcp].copy())
        ins["xmat"].append(d.site_xmat[tcp].copy())
        ins["jac"].append(np.vstack([d._jacp[:, :6], d._jacr[:, :6]]).reshape(36))
        ins["qvel"].append(d.qvel[:6].copy()); ins["bias"].append(d.qfrc_bias[:6].copy()); ins["ctrl"].append(u)
    for k, v in ins.items():
        out["pid_" + k] = np.array(v)

    # ---- C. pd_joint_ctrl via move_j (config_j gains)
    qpos_gains = {k: np.diag(v) for k, v in YML_J["qpos"].items()}
    N = 200
    pj = dict(q=[], v=[], target=[], u=[])
    for k in range(N):
        d = FakeData(md["nsite"], md["nbody"], md["nv"], md["nq"])
        d.qpos = rng.uniform(-3.3, 3.3, size=md["nq"]) if k % 5 == 0 else rng.uniform(-1.5, 1.5, size=md["nq"])
        d.qvel = rng.normal(size=md["nv"]) * 2
        target = np.concatenate([rng.uniform(-3.5, 3.5, 6) if k % 3 == 0 else d.qpos[:6] + rng.normal(size=6) * 0.3,
                                 [rng.uniform(0, 1)]])
        u = mvj.ctrl(0, fm, d, target, qpos_gains, np.zeros((1, 6)))
        pj["q"].append(d.qpos[:6].copy()); pj["v"].append(d.qvel[:6].copy()); pj["target"].append(target)
        pj["u"].append(u)
    for k, v in pj.items():
        out["movej_" + k] = np.array(v)
    out["movej_jnt_range"] = np.array(md["jnt_range"])[:6]
    out["movej_ctrl_range"] = np.array(md["act_ctrlrange"])[:7]

    # ---- D. move_l (pinv deltas through pd_joint_ctrl, config_l gains)
    pg = {k: np.diag(v) for k, v in YML_L["pos"].items()}
    rg = {k: np.diag(v) for k, v in YML_L["rot"].items()}
    N = 100
    ml = dict(q=[], v=[], traj=[], xpos=[], xmat=[], jacp=[], jacr=[], u=[], pinvp=[])
    for k in range(N):
        d = FakeData(md["nsite"], md["nbody"], md["nv"], md["nq"])
        d.qpos = rng.uniform(-1.5, 1.5, size=md["nq"])
        d.qvel = rng.normal(size=md["nv"])
        d.site_xpos[tcp] = rng.uniform([0.1, -0.2, 0.05], [0.5, 0.4, 0.4])
        d.site_xmat[tcp] = rand_rot(rng).reshape(9)
        d._jacp = rng.normal(size=(3, md["nv"])) * 0.3
        d._jacr = rng.normal(size=(3, md["nv"]))
        traj = np.concatenate([d.site_xpos[tcp] + rng.normal(size=3) * 0.05, rng.normal(size=3), [rng.uniform()]])
        u = mvl.ctrl(0, fm, d, traj, pg, rg, np.zeros((1, 3)), np.zeros((1, 3)))
        ml["q"].append(d.qpos[:6].copy()); ml["v"].append(d.qvel[:6].copy()); ml["traj"].append(traj)
        ml["xpos"].append(d.site_xpos[tcp].copy()); ml["xmat"].append(d.site_xmat[tcp].copy())
        ml["jacp"].append(d._jacp[:, :6].reshape(18)); ml["jacr"].append(d._jacr[:, :6].reshape(18))
        ml["u"].append(u); ml["pinvp"].append(np.linalg.pinv(d._jacp[:, :6]))
    for k, v in ml.items():
        out["movel_" + k] = np.array(v)

    # ---- E. trajectories
    starts = [np.array([0.29799994, 0.13349916, 0.1682003, -1.20920499, -1.20920054, 1.20920054, 0.0])]
    for _ in range(3):
        starts.append(np.concatenate([rng.uniform([0.2, 0.0, 0.1], [0.4, 0.3, 0.3]), rng.normal(size=3), [0.0]]))
    pp_rows, pp_dest, pp_shape = [], [], []
    for s in starts:
        pick = np.concatenate([rng.uniform([0.25, -0.1, 0.05], [0.35, 0.35, 0.06]), s[3:6], [0.5]])
        place = np.concatenate([[0.29799994, 0.25, 0.055111], s[3:6], [1.0]])
        place_in = place.copy()
        tr = bt.build_traj_l_pick_place(s.copy(), [pick.copy(), place_in], 120)
        pp_shape.append(tr.shape[0])
        assert np.all(tr.reshape(-1, 120, 7) == tr[::120][:, None, :])
        pp_rows.append(tr[::120])
        pp_dest.append(np.stack([pick, place]))
    out["pp_start"] = np.array(starts)
    out["pp_dest"] = np.array(pp_dest)
    out["pp_rows"] = np.array(pp_rows)
    out["pp_T"] = np.array(pp_shape)
    tj = []
    jstarts = [np.zeros(7), np.concatenate([rng.uniform(-1, 1, 6), [0]])]
    for s in jstarts:
        tr = bt.build_traj_j(s, 120)
        assert tr.shape == (60000, 7)
        assert np.all(tr.reshape(-1, 120, 7) == tr[::120][:, None, :])
        tj.append(tr[::120])
    out["trajj_start"] = np.array(jstarts)
    out["trajj_rows"] = np.array(tj)

    # ---- F. compute_reward
    N = 500
    obs_l, act_l, rew_l = [], [], []
    for k in range(N):
        o = rng.normal(size=24) * 0.2
        o[5] = rng.uniform(-0.05, 0.3)
        o[23] = float(rng.integers(0, 2))
        if k % 5 == 0:
            o[12:15] = rng.normal(size=3) * 0.02  # near place success
        if k % 7 == 0:
            o[9:12] = rng.normal(size=3) * 0.01
        a = np.concatenate([rng.uniform([0.05, -0.12, 0], [0.55, 0.38, 0.5]), [rng.uniform()]])
        r = UR3eEnv2.compute_reward(None, o, a)
        obs_l.append(o); act_l.append(a); rew_l.append(r)
    o = np.linspace(-0.3, 0.4, 24)
    o[23] = 1
    obs_l.append(o); act_l.append(np.array([0.3, 0.13, 0.1, 0.8]))
    rew_l.append(UR3eEnv2.compute_reward(None, o, act_l[-1]))
    out["rew_obs"], out["rew_act"], out["rew"] = np.array(obs_l), np.array(act_l), np.array(rew_l)

    # ---- G. predicates on synthetic contact lists
    cache = gu.init_collision_cache(fm)
    out["cache_gripper"] = np.array(sorted(cache[0]))
    out["cache_arm"] = np.array(sorted(cache[1]))
    ng = md["ngeom"]
    hnd = md["site_names"].index("handle_site")
    N = 400
    cg, cl, gs, rb, sc, tp, term, ptcp, phnd, pobs = [], [], [], [], [], [], [], [], [], []
    fish_g = md["geom_names"].index("fish")
    pad_g = [md["geom_names"].index(n) for n in ("left_pad1", "left_pad2", "right_pad1", "right_pad2")]
    for k in range(N):
        d = FakeData(md["nsite"], md["nbody"], md["nv"], md["nq"])
        nc = int(rng.integers(0, 10))
        pairs = []
        for _ in range(nc):
            if rng.uniform() < 0.5:
                pairs.append((int(rng.choice(pad_g)), fish_g) if rng.uniform() < 0.5 else (fish_g, int(rng.choice(pad_g))))
            else:
                pairs.append((int(rng.integers(0, ng)), int(rng.integers(0, ng))))
        d.contact = [_Obj(geom1=a, geom2=b) for a, b in pairs]
        d.ncon = nc
        d.site_xpos[hnd] = rng.uniform([0.2, -0.1, 0.0], [0.4, 0.3, 0.12])
        d.site_xpos[tcp] = d.site_xpos[hnd] + rng.normal(size=3) * (0.004 if k % 2 else 0.05)
        pl = np.zeros((10, 2), int)
        if nc:
            pl[:nc] = pairs
        cl.append(pl); cg.append(nc)
        gs.append(gu.get_block_grasp_state(fm, d))
        rb.append(gu.get_robust_block_grasp_state(fm, d))
        sc.append(gu.get_self_collision(fm, d, cache))
        tp.append(int(gu.get_mug_toppled(fm, d)))
        obs = np.zeros(24)
        obs[0:3] = d.site_xpos[tcp]
        obs[3:6] = d.site_xpos[hnd]
        if k % 9 == 0:
            obs[0:3] += 1.5
        fake_env = _Obj(model=fm, data=d, collision_cache=cache)
        with contextlib.redirect_stdout(io.StringIO()):
            term.append(int(UR3eEnv2._check_termination(fake_env, obs)))
        ptcp.append(d.site_xpos[tcp].copy()); phnd.append(d.site_xpos[hnd].copy()); pobs.append(obs)
    out["pred_ncon"] = np.array(cg)
    out["pred_pairs"] = np.array(cl)
    out["pred_grasp"] = np.array(gs)
    out["pred_robust"] = np.array(rb)
    out["pred_selfcol"] = np.array(sc)
    out["pred_toppled"] = np.array(tp)
    out["pred_term"] = np.array(term)
    out["pred_tcp"] = np.array(ptcp)
    out["pred_hnd"] = np.array(phnd)
    out["pred_obs"] = np.array(pobs)

    # ---- H. UR3eEnv (ur3e-v0) epilogue: compute_reward, _check_termination, get_table_collision
    #      on synthetic 13-d observations, actions in the v0 Box and contact lists
    lo0 = np.array([0.28799994, 0.13349916, 0.005, 0.0])
    hi0 = np.array([0.35799994, 0.35349916, 0.165, 1.0])
    table_g = md["geom_names"].index("table")
    arm_g = [md["geom_names"].index(n) for n in ("upperarm", "forearm", "wrist1", "wrist2", "wrist3", "collision")]
    N0 = 300
    v0_obs, v0_act, v0_rew, v0_term, v0_tab, v0_pairs, v0_ncon = [], [], [], [], [], [], []
    for k in range(N0):
        d = FakeData(md["nsite"], md["nbody"], md["nv"], md["nq"])
        nc = int(rng.integers(0, 8))
        pairs = []
        for _ in range(nc):
            u = rng.uniform()
            if u < 0.4:
                pairs.append((int(rng.choice(pad_g)), fish_g))
            elif u < 0.55:
                pairs.append((table_g, int(rng.choice(pad_g + arm_g))))
            elif u < 0.65:
                pairs.append((int(rng.choice(arm_g)), int(rng.choice(arm_g))))
            else:
                pairs.append((int(rng.integers(0, ng)), int(rng.integers(0, ng))))
        d.contact = [_Obj(geom1=a, geom2=b) for a, b in pairs]
        d.ncon = nc
        mug = rng.uniform([0.25, 0.05, 0.0], [0.36, 0.3, 0.2])
        if k % 7 == 0:
            mug = np.array([0.29799994, 0.25, 0.055111]) + rng.normal(size=3) * 0.003
        d.site_xpos[hnd] = mug
        g = mug + rng.normal(size=3) * (0.01 if k % 3 else 0.08)
        if k % 11 == 0:
            g = mug + np.array([1.2, 0.0, 0.0])
        if k % 4 == 0:  # gripper >= 0.5 above the block: the cubic height penalty vanishes
            g[2] = mug[2] + 0.5 + abs(rng.normal()) * 0.01
        d.site_xpos[tcp] = g
        pad = g + rng.normal(size=3) * 0.02
        obs = np.hstack([g, mug, [0.29799994, 0.25, 0.055111], [gu.get_block_grasp_state(fm, d)], pad])
        a = rng.uniform(lo0, hi0)
        fake_env = _Obj(model=fm, data=d, collision_cache=cache, t=k)
        with contextlib.redirect_stdout(io.StringIO()):
            v0_rew.append(UR3eEnv.compute_reward(fake_env, obs, a))
            v0_term.append(int(UR3eEnv._check_termination(fake_env, obs)))
        v0_tab.append(int(gu.get_table_collision(fm, d, cache)))
        pl = np.zeros((8, 2), int)
        if nc:
            pl[:nc] = pairs
        v0_pairs.append(pl); v0_ncon.append(nc)
        v0_obs.append(obs); v0_act.append(a)
    out["v0_obs"], out["v0_act"], out["v0_rew"] = np.array(v0_obs), np.array(v0_act), np.array(v0_rew)
    out["v0_term"], out["v0_table"] = np.array(v0_term), np.array(v0_tab)
    out["v0_pairs"], out["v0_ncon"] = np.array(v0_pairs), np.array(v0_ncon)

    # ---- I. augmented imitation trajectories (collect_demos.py:104-106), global np.random seeded per case
    aug_start, aug_dest, aug_seed, aug_idx, aug_rows = [], [], [], None, []
    for k, seed in enumerate([3, 1234]):
        s = np.array([0.29799994, 0.13349916, 0.1682003, -1.20920499, -1.20920054, 1.20920054, 0.0])
        s[:3] += rng.normal(size=3) * 0.01
        pick = np.concatenate([rng.uniform([0.29, 0.0, 0.05], [0.31, 0.14, 0.06]), s[3:6], [0.0]])
        place = np.concatenate([[0.29799994, 0.25, 0.055111], s[3:6], [1.0]])
        np.random.seed(seed)
        tr = bt.build_traj_l_pick_place_imitation_augmented(s.copy(), [pick.copy(), place.copy()], 120)
        assert tr.shape == (10500, 7)
        idx = sorted(set(range(0, 10500, 10)) | {j * 1500 + 1499 for j in range(7)} |
                     {j * 1500 + 999 for j in range(7)} | {j * 1500 + 1000 for j in range(7)})
        aug_idx = np.array(idx)
        aug_rows.append(tr[aug_idx])
        aug_start.append(s); aug_dest.append(np.stack([pick, place])); aug_seed.append(seed)
    out["aug_start"], out["aug_dest"], out["aug_seed"] = np.array(aug_start), np.array(aug_dest), np.array(aug_seed)
    out["aug_idx"], out["aug_rows"] = aug_idx, np.array(aug_rows)

    # ---- J. build_traj_l (build_traj.py:310-384: np.random.seed(49) cubic task-space path, hold from
    #      config_l.yml) and the config_l.yml gains move_l.main loads (move_l.py:93-95)
    tl = []
    lstarts = [np.array([0.29799994, 0.13349916, 0.1682003, -1.20920499, -1.20920054, 1.20920054, 0.0]),
               np.concatenate([rng.uniform([0.2, -0.1, 0.2], [0.4, 0.2, 0.5]), rng.normal(size=3), [0.0]])]
    for s in lstarts:
        tr = bt.build_traj_l(s.copy(), YML_L["hold"])
        assert tr.shape == (500 * YML_L["hold"], 7)
        assert np.all(tr.reshape(-1, YML_L["hold"], 7) == tr[::YML_L["hold"]][:, None, :])
        tl.append(tr[::YML_L["hold"]])
    out["trajl_start"], out["trajl_rows"], out["trajl_hold"] = np.array(lstarts), np.array(tl), np.array(YML_L["hold"])
    out["cfgl_pos"] = np.array([YML_L["pos"]["kp"], YML_L["pos"]["kd"]], dtype=np.float64)
    out["cfgl_rot"] = np.array([YML_L["rot"]["kp"], YML_L["rot"]["kd"]], dtype=np.float64)

    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "reference_golden.npz"), **out)
    meta = {"generator": "tools/make_golden.py", "reference": "derekc22/UR3e @ /root/reference",
            "scipy": __import__("scipy").__version__, "numpy": np.__version__,
            "keys": sorted(out.keys())}
    with open(os.path.join(OUT, "reference_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
