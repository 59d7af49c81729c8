"""ctypes front-end for the CPU oracle (oracle/_build/libur3e_oracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
bench.py `cpu_baseline` leg as the checker.  The product package (ur3e_amd)
never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libur3e_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB)
    return _lib


_SRCS = ("ur3e_oracle.c", "ur3e_oracle_batch.c", "ur3e_oracle_probe.c")


def build_native(out_dir: str) -> str:
    """Compile the oracle for THIS host's CPU (-O3 -march=native, contraction still off, so results
    are unchanged) into out_dir and return the .so path.  Used by bench.py's cpu_baseline leg on the
    GPU box, where the host CPU differs from the build container's."""
    os.makedirs(out_dir, exist_ok=True)
    so = os.path.join(out_dir, "libur3e_oracle_native.so")
    cc = os.environ.get("CC", "gcc")
    cmd = [cc, "-O3", "-march=native", "-fPIC", "-std=c99", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
           "-shared", "-o", so] + [os.path.join(_HERE, f) for f in _SRCS] + ["-lm"]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return so


def load_native(out_dir: str):
    L = ctypes.CDLL(build_native(out_dir))
    return L


class OracleConfig(ctypes.Structure):
    _fields_ = [
        ("task", ctypes.c_int), ("frame_skip", ctypes.c_int), ("max_episode_steps", ctypes.c_int),
        ("auto_reset", ctypes.c_int), ("reset_noise", ctypes.c_int), ("reset_key", ctypes.c_int),
        ("task_gains", ctypes.c_double * 12), ("joint_gains", ctypes.c_double * 12),
        ("seed", ctypes.c_ulonglong), ("env_id_offset", ctypes.c_int), ("envs_per_block", ctypes.c_int),
        ("tier_con_cap", ctypes.c_int), ("rot_joint_gains", ctypes.c_double * 12),
        ("np_chunk_lanes", ctypes.c_int), ("sensors", ctypes.c_int), ("schedule", ctypes.c_int),
    ]


def config_from(cfg) -> OracleConfig:
    """Copy a runtime.ConfigC (same field layout as ur3e_config_t) into an OracleConfig."""
    oc = OracleConfig()
    assert [f for f, _ in type(cfg)._fields_] == [f for f, _ in OracleConfig._fields_], "config layouts differ"
    ctypes.memmove(ctypes.byref(oc), ctypes.byref(cfg), ctypes.sizeof(OracleConfig))
    return oc


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleBatch:
    """N independent oracle envs with the same step semantics as ur3e_batch_step."""

    def __init__(self, model_c, cfg: OracleConfig, n_envs: int, L=None):
        self.L = lib() if L is None else L
        self.m = model_c
        self.cfg = cfg
        self.n = n_envs
        self.nq, self.nv = model_c.nq, model_c.nv
        self.buf = ctypes.create_string_buffer(self.L.ur3o_sizeof_env() * n_envs)
        self.od = self.L.ur3o_obs_dim(ctypes.c_int(cfg.task))
        self.obs = np.zeros((n_envs, self.od))
        self.L.ur3o_batch_init(ctypes.byref(self.m), ctypes.byref(self.cfg), ctypes.c_int(n_envs), self.buf,
                               _p(self.obs))

    def reset_all(self):
        """reset every env again (a new episode: fresh reset noise), as ur3e_batch_reset(mask=None)"""
        obs = np.zeros((self.n, self.od))
        sz = self.L.ur3o_sizeof_env()
        for i in range(self.n):
            ptr = ctypes.cast(ctypes.addressof(self.buf) + sz * i, ctypes.c_void_p)
            self.L.ur3o_batch_reset_one(ctypes.byref(self.m), ctypes.byref(self.cfg), ptr, _p(obs[i]))
        self.obs = obs
        return obs

    def step(self, actions: np.ndarray):
        actions = np.ascontiguousarray(actions, dtype=np.float64)
        n = self.n
        obs = np.zeros((n, self.od))
        rew = np.zeros(n)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        tobs = np.zeros((n, self.od))
        self.L.ur3o_batch_step(ctypes.byref(self.m), ctypes.byref(self.cfg), ctypes.c_int(n), self.buf,
                               _p(actions), ctypes.c_int(actions.shape[1]), _p(obs), _p(rew), _p(term),
                               _p(trunc), _p(tobs))
        self.obs = obs
        return obs, rew, term, trunc, tobs

    def get_state(self):
        qp = np.zeros((self.n, self.nq))
        qv = np.zeros((self.n, self.nv))
        wa = np.zeros((self.n, self.nv))
        nc = np.zeros(self.n, np.int32)
        self.L.ur3o_batch_get_state(ctypes.byref(self.m), ctypes.c_int(self.n), self.buf, _p(qp), _p(qv), _p(wa),
                                    _p(nc))
        return qp, qv, wa, nc

    def set_state(self, qpos, qvel, warm=None):
        qpos = np.ascontiguousarray(qpos, dtype=np.float64)
        qvel = np.ascontiguousarray(qvel, dtype=np.float64)
        warm = None if warm is None else np.ascontiguousarray(warm, dtype=np.float64)
        self.L.ur3o_batch_set_state(ctypes.byref(self.m), ctypes.c_int(self.n), self.buf, _p(qpos), _p(qvel),
                                    _p(warm))

    def sensordata(self):
        """[n, nsensordata] mjData.sensordata of every env's last forward"""
        nsd = self.m.nsensordata
        out = np.zeros((self.n, max(nsd, 1)))
        sz = self.L.ur3o_sizeof_env()
        for i in range(self.n):
            ptr = ctypes.cast(ctypes.addressof(self.buf) + sz * i, ctypes.c_void_p)
            self.L.ur3o_env_sensordata(ctypes.byref(self.m), ptr, _p(out[i]))
        return out[:, :nsd]

    def _env_ptr(self, i):
        return ctypes.cast(ctypes.addressof(self.buf) + self.L.ur3o_sizeof_env() * i, ctypes.c_void_p)

    def task_space_state(self, touch_left: int, touch_right: int):
        """[n, 7] controller_func.get_task_space_state of every env's last forward: tcp xpos, tcp rotvec
        (scipy from_matrix(...).as_rotvec()), boolean grasp contact (touch columns left / right)"""
        out = np.zeros((self.n, 7))
        for i in range(self.n):
            self.L.ur3o_env_task_space_state(ctypes.byref(self.m), self._env_ptr(i), ctypes.c_int(touch_left),
                                             ctypes.c_int(touch_right), _p(out[i]))
        return out

    def actuator_force(self):
        """[n, nu] mjData.actuator_force of every env's last forward (get_jnt_torques)"""
        out = np.zeros((self.n, self.m.nu))
        for i in range(self.n):
            self.L.ur3o_env_actuator_force(ctypes.byref(self.m), self._env_ptr(i), _p(out[i]))
        return out

    def get_ctrl(self):
        """[n, nu] d.ctrl applied by every env's last step"""
        nu = self.m.nu
        return np.stack([self.diag(i)["ctrl"][:nu] for i in range(self.n)])

    def diag(self, i):
        ncon, nefc, nit = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        touch = np.zeros(4)
        sz = self.L.ur3o_sizeof_env()
        ptr = ctypes.cast(ctypes.addressof(self.buf) + sz * i, ctypes.c_void_p)
        self.L.ur3o_env_diag(ptr, ctypes.byref(ncon), ctypes.byref(nefc), ctypes.byref(nit), _p(touch))
        ctrl = np.zeros(8)
        self.L.ur3o_env_ctrl(ptr, _p(ctrl))
        return dict(ncon=ncon.value, nefc=nefc.value, niter=nit.value, touch=touch, ctrl=ctrl)


def forward_state(model_c, qpos, qvel=None):
    L = lib()
    nq, nv, ns = model_c.nq, model_c.nv, model_c.nsite
    qpos = np.ascontiguousarray(qpos, dtype=np.float64)
    qvel = np.zeros(nv) if qvel is None else np.ascontiguousarray(qvel, dtype=np.float64)
    sx = np.zeros((max(ns, 1), 3))
    sm = np.zeros((max(ns, 1), 9))
    bias = np.zeros(nv)
    M = np.zeros((nv, nv))
    ncon = ctypes.c_int()
    L.ur3o_forward_state(ctypes.byref(model_c), _p(qpos), _p(qvel), _p(sx), _p(sm), _p(bias), _p(M),
                         ctypes.byref(ncon))
    return dict(site_xpos=sx, site_xmat=sm, qfrc_bias=bias, qM=M, ncon=ncon.value)


def v0_epilogue(model_c, pairs, obs13, act4):
    """ur3e-v0 reward / termination / table collision for a synthetic contact list."""
    L = lib()
    pairs = np.asarray(pairs, dtype=np.int32).reshape(-1, 2)
    g1 = np.ascontiguousarray(pairs[:, 0])
    g2 = np.ascontiguousarray(pairs[:, 1])
    r = ctypes.c_double()
    oi = np.zeros(2, np.int32)
    L.ur3o_v0_epilogue(ctypes.byref(model_c), ctypes.c_int(len(pairs)), _p(g1), _p(g2),
                       _p(np.ascontiguousarray(obs13, dtype=np.float64)),
                       _p(np.ascontiguousarray(act4, dtype=np.float64)), ctypes.byref(r), _p(oi))
    return r.value, int(oi[0]), int(oi[1])


def rotvec_from_matrix(xmat):
    """scipy Rotation.from_matrix(xmat).as_rotvec() as the oracle restates it (utils/utils.py:158-162)"""
    L = lib()
    xmat = np.ascontiguousarray(xmat, dtype=np.float64).reshape(9)
    out = np.zeros(3)
    L.ur3o_rotvec_from_matrix(_p(xmat), _p(out))
    return out


def rot_err(xmat, target):
    L = lib()
    xmat = np.ascontiguousarray(xmat, dtype=np.float64).reshape(9)
    target = np.ascontiguousarray(target, dtype=np.float64)
    out = np.zeros(3)
    L.ur3o_rot_err(_p(xmat), _p(target), _p(out))
    return out


def pid_task_ctrl_raw(traj7, tcp_xpos, tcp_xmat, jac_arm, qvel6, bias6, gains12, grip_scale=255.0):
    L = lib()

    class TG(ctypes.Structure):
        _fields_ = [("g", ctypes.c_double * 12)]

    tg = TG()
    for k in range(12):
        tg.g[k] = gains12[k]
    a = [np.ascontiguousarray(x, dtype=np.float64).reshape(-1) for x in (traj7, tcp_xpos, tcp_xmat, jac_arm, qvel6, bias6)]
    out = np.zeros(7)
    L.ur3o_pid_task_ctrl_raw(*[_p(x) for x in a], ctypes.byref(tg), ctypes.c_double(grip_scale), _p(out))
    return out


def pd_joint_ctrl_raw(q6, v6, delta6, jnt_range12, ctrl_range12, kp6, kd6):
    L = lib()
    g = np.ascontiguousarray(np.concatenate([kp6, kd6]), dtype=np.float64)
    a = [np.ascontiguousarray(x, dtype=np.float64).reshape(-1) for x in (q6, v6, delta6, jnt_range12, ctrl_range12)]
    out = np.zeros(6)
    L.ur3o_pd_joint_ctrl_raw(*[_p(x) for x in a], _p(g), _p(out))
    return out


def move_l_ctrl_raw(traj7, tcp_xpos, tcp_xmat, jacp_arm, jacr_arm, q6, v6, jnt_range12, ctrl_range12,
                    pos_kp, pos_kd, rot_kp, rot_kd, grip_scale=255.0):
    L = lib()
    gp = np.ascontiguousarray(np.concatenate([pos_kp, pos_kd]), dtype=np.float64)
    gr = np.ascontiguousarray(np.concatenate([rot_kp, rot_kd]), dtype=np.float64)
    a = [np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
         for x in (traj7, tcp_xpos, tcp_xmat, jacp_arm, jacr_arm, q6, v6, jnt_range12, ctrl_range12)]
    out = np.zeros(7)
    L.ur3o_move_l_ctrl_raw(*[_p(x) for x in a], _p(gp), _p(gr), ctypes.c_double(grip_scale), _p(out))
    return out


def pinv3x6(J):
    L = lib()
    J = np.ascontiguousarray(J, dtype=np.float64).reshape(18)
    P = np.zeros(18)
    L.ur3o_pinv3x6(_p(J), _p(P))
    return P.reshape(6, 3)


def reward_v2(obs, act):
    L = lib()
    L.ur3o_reward_v2.restype = ctypes.c_double
    o = np.ascontiguousarray(obs, dtype=np.float64)
    a = np.ascontiguousarray(act, dtype=np.float64)
    return L.ur3o_reward_v2(_p(o), _p(a))


def philox(ctr, key):
    L = lib()
    c = (ctypes.c_uint * 4)(*ctr)
    k = (ctypes.c_uint * 2)(*key)
    o = (ctypes.c_uint * 4)()
    L.ur3o_philox4x32(c, k, o)
    return list(o)


class OracleData:
    """One oracle mjData-like record (ur3o_data) for the physics known-answer and independent-solver
    tests: set qpos/qvel/ctrl, run ur3o_forward / ur3o_step, read state, contacts and constraint rows
    (oracle/ur3e_oracle_probe.c)."""

    MAXC, MAXR = 64, 256

    def __init__(self, model_c, L=None):
        self.L = lib() if L is None else L
        self.m = model_c
        self.nq, self.nv, self.nu = model_c.nq, model_c.nv, model_c.nu
        self.buf = ctypes.create_string_buffer(self.L.ur3o_sizeof_data())
        self.L.ur3o_data_init(ctypes.byref(self.m), self.buf)

    def set(self, qpos=None, qvel=None, ctrl=None, warm=None):
        a = [None if x is None else np.ascontiguousarray(x, dtype=np.float64) for x in (qpos, qvel, ctrl)]
        self.L.ur3o_data_set(ctypes.byref(self.m), self.buf, *[_p(x) for x in a])
        if warm is not None:
            w = np.ascontiguousarray(warm, dtype=np.float64)
            self.L.ur3o_data_set_warmstart(ctypes.byref(self.m), self.buf, _p(w))

    def forward(self):
        self.L.ur3o_forward(ctypes.byref(self.m), self.buf)

    def step(self, n=1):
        for _ in range(n):
            self.L.ur3o_step(ctypes.byref(self.m), self.buf)

    def state(self):
        nv = self.nv
        out = dict(qpos=np.zeros(self.nq), qvel=np.zeros(nv), qacc=np.zeros(nv), qacc_smooth=np.zeros(nv),
                   qfrc_smooth=np.zeros(nv), qM=np.zeros((nv, nv)))
        self.L.ur3o_data_get(ctypes.byref(self.m), self.buf, *[_p(out[k]) for k in
                                                                ("qpos", "qvel", "qacc", "qacc_smooth",
                                                                 "qfrc_smooth", "qM")])
        out["niter"] = self.L.ur3o_data_niter(self.buf)
        return out

    def sensordata(self):
        out = np.zeros(max(self.m.nsensordata, 1))
        self.L.ur3o_data_sensordata(ctypes.byref(self.m), self.buf, _p(out))
        return out[:self.m.nsensordata]

    def rnepost(self):
        nb = self.m.nbody
        out = {k: np.zeros((nb, 6)) for k in ("cacc", "cfrc_int", "cfrc_ext")}
        self.L.ur3o_data_rnepost(ctypes.byref(self.m), self.buf, _p(out["cacc"]), _p(out["cfrc_int"]),
                                 _p(out["cfrc_ext"]))
        return out

    def contacts(self):
        C = self.MAXC
        pos, frame, dist = np.zeros((C, 3)), np.zeros((C, 9)), np.zeros(C)
        geoms, fr, mu, adr = np.zeros((C, 2), np.int32), np.zeros((C, 5)), np.zeros(C), np.zeros(C, np.int32)
        n = self.L.ur3o_data_contacts(self.buf, C, _p(pos), _p(frame), _p(dist), _p(geoms), _p(fr), _p(mu), _p(adr))
        n = min(n, C)
        return dict(n=n, pos=pos[:n], frame=frame[:n].reshape(n, 3, 3), dist=dist[:n], geoms=geoms[:n],
                    friction=fr[:n], mu=mu[:n], efc_address=adr[:n])

    def efc(self):
        R_, nv = self.MAXR, self.nv
        ints = {k: np.zeros(R_, np.int32) for k in ("type", "id", "state")}
        J = np.zeros((R_, nv))
        dbl = {k: np.zeros(R_) for k in ("pos", "margin", "frictionloss", "diagApprox", "R", "D", "vel", "aref",
                                          "force")}
        n = self.L.ur3o_data_efc(ctypes.byref(self.m), self.buf, R_, _p(ints["type"]), _p(ints["id"]),
                                 _p(ints["state"]), _p(J), *[_p(dbl[k]) for k in
                                                             ("pos", "margin", "frictionloss", "diagApprox", "R",
                                                              "D", "vel", "aref", "force")])
        n = min(n, R_)
        out = {k: v[:n] for k, v in ints.items()}
        out.update({k: v[:n] for k, v in dbl.items()})
        out["J"] = J[:n]
        out["n"] = n
        return out
