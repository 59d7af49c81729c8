"""Host-side binding of the MI355X C ABI (include/ur3e_batch.h).

`Batch` owns one `ur3e_batch_t` handle: N environments resident in HBM on one
GPU.  Buffers exchanged with the library are torch tensors on that device; all
calls enqueue on torch's current stream, so torch events time them and torch
ops consume the results without host round-trips.

There is no CPU fallback: if the HIP library or a GPU is missing this module
raises.  (The CPU oracle in oracle/ is test infrastructure and is never used
here.)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .model.compiler import UR3eModelC, load_json, to_ctypes

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UR3E_LIB", os.path.join(_HERE, "_lib", "libur3e_amd.so"))
ASSETS = os.path.join(_HERE, "assets")

TASK_GYM_V2, TASK_TRAJ_L, TASK_MOVE_J, TASK_CTRL = 0, 1, 2, 3
TASK_GYM_V0, TASK_IMIT_INDIRECT, TASK_IMIT_DIRECT = 4, 5, 6
TASK_MOVE_L = 7

# controller/config/config_l_mug.yml (used by UR3eEnv2, ur3e_env2.py:66-68)
GAINS_L_MUG = dict(kp_pos=[220.0, 220.0, 120.0], kd_pos=[20.0, 20.0, 40.0],
                   kp_rot=[35.0, 15.0, 15.0], kd_rot=[2.0, 2.0, 2.0])
# gymnasium_env/envs/ur3e_env.py:49-55 (UR3eEnv, ur3e-v0)
GAINS_V0 = dict(kp_pos=[320.0, 320.0, 320.0], kd_pos=[20.0, 20.0, 25.0],
                kp_rot=[325.0, 325.0, 325.0], kd_rot=[2.0, 2.0, 2.0])
# controller/config/config_j.yml (move_j)
GAINS_J = dict(kp=[20.0, 380.0, 300.0, 20.0, 30.0, 10.0], kd=[5.0] * 6)
# controller/config/config_l.yml (move_l: "pos" and "rot" joint-space PD gains)
GAINS_L_POS = dict(kp=[20.0, 60.0, 20.0, 20.0, 20.0, 10.0], kd=[5.0, 15.0, 5.0, 5.0, 5.0, 20.0])
GAINS_L_ROT = dict(kp=[5.02, 5.01, 5.80, 5.80, 5.09, 5.80], kd=[5.0, 50.0, 10.0, 5.0, 5.0, 5.0])

_lib = None
_libs = {}  # other builds of the library loaded side by side (diagnostic variants), by path


class ConfigC(ctypes.Structure):
    _fields_ = [
        ("task", ctypes.c_int), ("frame_skip", ctypes.c_int), ("max_episode_steps", ctypes.c_int),
        ("auto_reset", ctypes.c_int), ("reset_noise", ctypes.c_int), ("reset_key", ctypes.c_int),
        ("task_gains", ctypes.c_double * 12), ("joint_gains", ctypes.c_double * 12),
        ("seed", ctypes.c_ulonglong), ("env_id_offset", ctypes.c_int), ("envs_per_block", ctypes.c_int),
        ("tier_con_cap", ctypes.c_int), ("rot_joint_gains", ctypes.c_double * 12),
        ("np_chunk_lanes", ctypes.c_int), ("sensors", ctypes.c_int), ("schedule", ctypes.c_int),
    ]


def load_library(path: str | None = None):
    """Load the in-tree HIP library (or, given `path`, another build of it, e.g. a diagnostic variant,
    side by side with the product library); raise loudly when it is absent."""
    global _lib
    if path is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        path = os.path.abspath(path)
        if path not in _libs:
            if not os.path.exists(path):
                raise RuntimeError(f"MI355X library variant missing: {path}")
            _libs[path] = _bind(ctypes.CDLL(path))
        return _libs[path]
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"MI355X library missing: {LIB_PATH} (run __graft_entry__.build())")
    _lib = _bind(ctypes.CDLL(LIB_PATH))
    return _lib


def _bind(L):
    vp, ip, dp = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    L.ur3e_last_error.restype = ctypes.c_char_p
    L.ur3e_batch_create.argtypes = [vp, vp, ip, ip, ctypes.POINTER(vp)]
    L.ur3e_batch_destroy.argtypes = [vp]
    L.ur3e_batch_reset.argtypes = [vp, vp, vp, vp]
    L.ur3e_batch_step.argtypes = [vp, vp, ip, vp, vp, vp, vp, vp, vp]
    L.ur3e_batch_get_state.argtypes = [vp, vp, vp, vp, vp]
    L.ur3e_batch_set_state.argtypes = [vp, vp, vp, vp, vp]
    L.ur3e_batch_get_info.argtypes = [vp, vp, vp, vp, vp, vp]
    L.ur3e_batch_last_step_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.ur3e_batch_set_timing.argtypes = [vp, ip]
    L.ur3e_batch_overflow_count.argtypes = [vp, ctypes.POINTER(ctypes.c_ulonglong)]
    L.ur3e_batch_tier_counts.argtypes = [vp, ctypes.POINTER(ctypes.c_ulonglong)]
    L.ur3e_batch_set_queue_split.argtypes = [vp, ctypes.c_int]
    L.ur3e_batch_get_touch.argtypes = [vp, vp, vp]
    L.ur3e_batch_get_carry.argtypes = [vp, vp, vp]
    L.ur3e_batch_get_ctrl.argtypes = [vp, vp, vp]
    L.ur3e_batch_get_sensordata.argtypes = [vp, vp, vp]
    L.ur3e_batch_get_task_space_state.argtypes = [vp, vp, vp]
    L.ur3e_batch_get_actuator_force.argtypes = [vp, vp, vp]
    L.ur3e_batch_queue_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_ulonglong)]
    L.ur3e_batch_mid_count.argtypes = [vp, ctypes.POINTER(ctypes.c_ulonglong)]
    L.ur3e_batch_set_queue_debug.argtypes = [vp, ctypes.c_uint, ip]
    L.ur3e_debug_hold_slots.argtypes = [ip, ip, ip, vp, ctypes.POINTER(ip)]
    L.ur3e_batch_tier_kernel.argtypes = [vp, ip, ctypes.POINTER(ip), ctypes.POINTER(ip), ctypes.POINTER(ip),
                                         ctypes.c_char_p, ip, ctypes.c_char_p, ip]
    for f in ("ur3e_batch_num_envs", "ur3e_batch_nq", "ur3e_batch_nv", "ur3e_batch_nu", "ur3e_batch_obs_dim",
              "ur3e_batch_schedule"):
        getattr(L, f).argtypes = [vp]
    del dp
    return L


def hold_slots(workgroups: int, hold_us: int, stream=None, device: int = 0) -> int:
    """Diagnostic: occupy most workgroup slots of the GPU for hold_us microseconds (ur3e_debug_hold_slots)
    on `stream` (a torch stream; default: torch's current stream); returns once they are all resident,
    with the number that had started."""
    import torch
    L = load_library()
    st = (stream or torch.cuda.current_stream(device)).cuda_stream
    started = ctypes.c_int()
    _check(L.ur3e_debug_hold_slots(device, workgroups, hold_us, ctypes.c_void_p(st), ctypes.byref(started)), L)
    return started.value


def _check(rc, L=None):
    if rc != 0:
        L = L or _lib
        raise RuntimeError(f"ur3e library error {rc}: {L.ur3e_last_error().decode()}")


def load_model(name: str = "main"):
    """Compiled model dict + C image for one of the reference models (main, ur3e_2f85, ur3e_raw)."""
    md = load_json(os.path.join(ASSETS, f"{name}.model.json"))
    return md, to_ctypes(md)


def make_config(task=TASK_GYM_V2, frame_skip=2, max_episode_steps=2500, auto_reset=True, reset_noise=True,
                reset_key=None, model=None, seed=0, env_id_offset=0, envs_per_block=0,
                task_gains=None, joint_gains=None, tier_con_cap=0, rot_joint_gains=None,
                np_chunk_lanes=0, sensors=False, schedule=0, config_yaml_path=None) -> ConfigC:
    c = ConfigC()
    c.task = task
    c.frame_skip = frame_skip
    c.max_episode_steps = max_episode_steps
    c.auto_reset = int(auto_reset)
    # True/1: "high" (ur3e-v2); 2 "med"; 3 "low"; also accepts the reference's names
    c.reset_noise = {"high": 1, "med": 2, "low": 3, None: 0, "deterministic": 0}.get(reset_noise, None) \
        if (reset_noise is None or isinstance(reset_noise, str)) else int(reset_noise)
    if reset_key is None:
        reset_key = model["id_key_down"] if model is not None else -1
    c.reset_key = reset_key
    tg = task_gains or GAINS_L_MUG
    g = list(tg["kp_pos"]) + list(tg["kd_pos"]) + list(tg["kp_rot"]) + list(tg["kd_rot"])
    if (joint_gains is None or rot_joint_gains is None) and task in (TASK_MOVE_J, TASK_MOVE_L):
        # the reference's drivers read their gains from the YAML configs (move_j.py:46-52: config_j.yml;
        # move_l.py:92-99: config_l.yml, pos and rot sections), from the cwd as it does, else the packaged copies
        from . import gains as _gains
        if task == TASK_MOVE_J:
            joint_gains = joint_gains or _gains.joint_gains(config_yaml_path)
        else:
            mpos, mrot = _gains.move_l_gains(config_yaml_path)
            joint_gains = joint_gains or mpos
            rot_joint_gains = rot_joint_gains or mrot
    jg = joint_gains or (GAINS_L_POS if task == TASK_MOVE_L else GAINS_J)
    j = list(jg["kp"]) + list(jg["kd"])
    rg = rot_joint_gains or GAINS_L_ROT
    r = list(rg["kp"]) + list(rg["kd"])
    for k in range(12):
        c.task_gains[k] = g[k]
        c.joint_gains[k] = j[k]
        c.rot_joint_gains[k] = r[k]
    c.seed = seed
    c.env_id_offset = env_id_offset
    c.envs_per_block = envs_per_block
    c.tier_con_cap = tier_con_cap
    c.np_chunk_lanes = np_chunk_lanes
    c.sensors = int(sensors)
    c.schedule = int(schedule)
    return c


def action_dim(task: int, nu: int) -> int:
    """Width of one env's action row for a task (what ur3e_batch_step checks `adim` against)."""
    if task in (TASK_GYM_V2, TASK_GYM_V0, TASK_IMIT_INDIRECT):
        return 4
    if task in (TASK_CTRL, TASK_IMIT_DIRECT):
        return nu
    return 7


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Batch:
    """N UR3e environments on one GPU (C ABI handle + device tensors)."""

    def __init__(self, model_c: UR3eModelC, cfg: ConfigC, n_envs: int, device: int = 0, lib: str | None = None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("ur3e_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.torch = torch
        self.L = load_library(lib)
        self.device = torch.device("cuda", device)
        self.model_c = model_c
        self.cfg = cfg
        self.n = n_envs
        self.nq, self.nv, self.nu = model_c.nq, model_c.nv, model_c.nu
        h = ctypes.c_void_p()
        torch.cuda.set_device(self.device)
        self._chk(self.L.ur3e_batch_create(ctypes.byref(model_c), ctypes.byref(cfg), n_envs, device, ctypes.byref(h)))
        self.h = h
        f64 = dict(dtype=torch.float64, device=self.device)
        self.obs_dim = self.L.ur3e_batch_obs_dim(h)
        self.act_dim = action_dim(cfg.task, self.nu)
        self.obs = torch.zeros((n_envs, self.obs_dim), **f64)
        self.reward = torch.zeros(n_envs, **f64)
        self.terminated = torch.zeros(n_envs, dtype=torch.uint8, device=self.device)
        self.truncated = torch.zeros(n_envs, dtype=torch.uint8, device=self.device)
        self.terminal_obs = torch.zeros((n_envs, self.obs_dim), **f64)
        self.reset()

    @staticmethod
    def torch_ptr(t):
        """device pointer of a contiguous tensor (or a contiguous row view of one)"""
        if not t.is_contiguous():
            raise ValueError("ur3e_amd: tensor must be contiguous")
        return _ptr(t)

    def out_ptr(self, out, cols: int, what: str):
        """device pointer of a caller-provided output buffer the kernels fill with n x cols doubles:
        checked for device, dtype, shape and contiguity before any launch (a wrong buffer would be
        written out of bounds on the device)"""
        t = self.torch
        if not isinstance(out, t.Tensor):
            raise ValueError(f"{what}: out must be a torch tensor")
        if out.device != self.device:
            raise ValueError(f"{what}: out is on {out.device}, the batch on {self.device}")
        if out.dtype != t.float64:
            raise ValueError(f"{what}: out must be float64, got {out.dtype}")
        if tuple(out.shape) != (self.n, cols):
            raise ValueError(f"{what}: out must have shape ({self.n}, {cols}), got {tuple(out.shape)}")
        if not out.is_contiguous():
            raise ValueError(f"{what}: out must be contiguous")
        return _ptr(out)

    def _chk(self, rc):
        _check(rc, self.L)

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "h", None):
            self.L.ur3e_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, mask=None):
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=self.torch.uint8).contiguous()
        self._chk(self.L.ur3e_batch_reset(self.h, _ptr(m), _ptr(self.obs), self._stream()))
        return self.obs

    def step(self, actions, out=None):
        """One env-step of every env.  `out` = (obs [n, obs_dim] f64, reward [n] f64, terminated [n] u8,
        truncated [n] u8) device tensors the library writes instead of the handle's own buffers (e.g. views
        of one payload a collective then sends whole); each is checked before the launch."""
        a = actions.to(device=self.device, dtype=self.torch.float64).contiguous()
        if out is None:
            obs, rew, term, trunc = self.obs, self.reward, self.terminated, self.truncated
        else:
            obs, rew, term, trunc = out
            t = self.torch
            for x, shape, dt, what in ((obs, (self.n, self.obs_dim), t.float64, "obs"), (rew, (self.n,), t.float64, "reward"),
                                       (term, (self.n,), t.uint8, "terminated"), (trunc, (self.n,), t.uint8, "truncated")):
                if not isinstance(x, t.Tensor) or x.device != self.device or x.dtype != dt or tuple(x.shape) != shape \
                        or not x.is_contiguous():
                    raise ValueError(f"step: out {what} must be a contiguous {dt} tensor of shape {shape} on {self.device}")
        self._chk(self.L.ur3e_batch_step(self.h, _ptr(a), a.shape[1], _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc),
                                      _ptr(self.terminal_obs), self._stream()))
        return obs, rew, term, trunc, self.terminal_obs

    def get_state(self):
        t = self.torch
        qp = t.empty((self.n, self.nq), dtype=t.float64, device=self.device)
        qv = t.empty((self.n, self.nv), dtype=t.float64, device=self.device)
        wa = t.empty((self.n, self.nv), dtype=t.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_state(self.h, _ptr(qp), _ptr(qv), _ptr(wa), self._stream()))
        return qp, qv, wa

    def set_state(self, qpos, qvel, warm=None):
        t = self.torch
        qp = t.as_tensor(qpos, dtype=t.float64).to(self.device).contiguous()
        qv = t.as_tensor(qvel, dtype=t.float64).to(self.device).contiguous()
        wa = None if warm is None else t.as_tensor(warm, dtype=t.float64).to(self.device).contiguous()
        self._chk(self.L.ur3e_batch_set_state(self.h, _ptr(qp), _ptr(qv), _ptr(wa), self._stream()))

    def get_info(self):
        t = self.torch
        nc = t.empty(self.n, dtype=t.int32, device=self.device)
        el = t.empty(self.n, dtype=t.int32, device=self.device)
        er = t.empty(self.n, dtype=t.float64, device=self.device)
        nw = t.empty(self.n, dtype=t.int32, device=self.device)
        self._chk(self.L.ur3e_batch_get_info(self.h, _ptr(nc), _ptr(el), _ptr(er), _ptr(nw), self._stream()))
        return dict(ncon=nc, ep_len=el, ep_return=er, nwarn=nw)

    def get_ctrl(self):
        """[N, nu] d.ctrl applied by the last step."""
        out = self.torch.empty((self.n, self.nu), dtype=self.torch.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_ctrl(self.h, _ptr(out), self._stream()))
        return out

    def get_sensordata(self):
        """[N, nsensordata] mjData.sensordata of the last forward (config sensors=True), in the model's
        sensor declaration order (sensor_names / sensor_adr of the model dict)"""
        nsd = self.model_c.nsensordata
        out = self.torch.zeros((self.n, max(nsd, 1)), dtype=self.torch.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_sensordata(self.h, _ptr(out), self._stream()))
        return out[:, :nsd]

    def get_task_space_state(self):
        """[N, 7] controller_func.get_task_space_state of the last step: tcp xpos, tcp rotvec (scipy
        from_matrix(...).as_rotvec() restated), boolean grasp contact -- computed on the device"""
        out = self.torch.empty((self.n, 7), dtype=self.torch.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_task_space_state(self.h, _ptr(out), self._stream()))
        return out

    def get_actuator_force(self, out=None):
        """[N, nu] mjData.actuator_force of the last forward (get_jnt_torques); `out` may be a row view
        of a recording buffer"""
        if out is None:
            out = self.torch.empty((self.n, self.nu), dtype=self.torch.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_actuator_force(self.h, self.out_ptr(out, self.nu, "get_actuator_force"),
                                                       self._stream()))
        return out

    def get_carry(self):
        """[N, 54] stale-kinematics snapshot: tcp xpos(3), xmat(9), arm Jacobian 6x6, qfrc_bias[0:6]."""
        out = self.torch.empty((self.n, 54), dtype=self.torch.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_carry(self.h, _ptr(out), self._stream()))
        return out

    def touch_index(self, side: str) -> int:
        """Column of get_touch() for the left / right pad sensor (site on the lpad / rpad body)."""
        body = self.model_c.id_body_lpad if side == "left" else self.model_c.id_body_rpad
        for k in range(self.model_c.ntouch):
            if self.model_c.site_bodyid[self.model_c.touch_site[k]] == body:
                return k
        raise KeyError(side)

    def get_touch(self):
        """Touch sensors [N, ntouch] after the last forward (mjSENS_TOUCH on the pad sites)."""
        nt = max(self.model_c.ntouch, 1)
        out = self.torch.zeros((self.n, nt), dtype=self.torch.float64, device=self.device)
        self._chk(self.L.ur3e_batch_get_touch(self.h, _ptr(out), self._stream()))
        return out[:, :self.model_c.ntouch]

    def tier_counts(self) -> tuple:
        """Since create: (env-steps the compact tier handed on -- to the grasp tier while routing is in
        use, else straight to the full-capacity tier --, env-steps that reached the full-capacity tier,
        env-steps routed straight to the grasp tier)."""
        v = (ctypes.c_ulonglong * 3)()
        self._chk(self.L.ur3e_batch_tier_counts(self.h, v))
        return int(v[0]), int(v[1]), int(v[2])

    def mid_count(self) -> int:
        """Since create: env-steps routed to the mid tier (16 contacts / 64 rows, between the compact and the
        grasp tier); its bails are counted again in tier_counts()[2]."""
        v = ctypes.c_ulonglong()
        self._chk(self.L.ur3e_batch_mid_count(self.h, ctypes.byref(v)))
        return int(v.value)

    def queue_stats(self) -> tuple:
        """Since create, substep work queue: (units that gave up waiting for their producer, static first
        units claimed and run by their consumer)."""
        v = (ctypes.c_ulonglong * 2)()
        self._chk(self.L.ur3e_batch_queue_stats(self.h, v))
        return int(v[0]), int(v[1])

    def set_queue_split(self, percent: int):
        """Substep work queue: the last `percent` % of each queue's envs run their last substep as two half
        units (include/ur3e_batch.h: ur3e_batch_set_queue_split); results never change."""
        self._chk(self.L.ur3e_batch_set_queue_split(self.h, int(percent)))

    def set_queue_debug(self, spin_limit: int = 0, leave_static_units: bool = False):
        """Diagnostics of the substep queue: flag polls before a waiting unit gives up (0 = built-in
        bound); leave_static_units: workgroups skip their static first units (consumers claim them)."""
        self._chk(self.L.ur3e_batch_set_queue_debug(self.h, int(spin_limit), int(leave_static_units)))

    def overflow_count(self) -> int:
        """Env-steps the compact tier handed to the full-capacity tier since create."""
        v = ctypes.c_ulonglong()
        self._chk(self.L.ur3e_batch_overflow_count(self.h, ctypes.byref(v)))
        return int(v.value)

    TIERS = {"step": 0, "compact": 0, "grasp": 1, "full": 2, "mid": 3}

    def kernel_info(self, tier="step") -> dict:
        """The kernel this handle launches for `tier` ("step"/"compact": the dominant step kernel; "mid"; "grasp";
        "full": the full-capacity fallback), as the library picks it (ur3e_batch_tier_kernel): envs
        resident per CU, LDS bytes per workgroup, registers per lane, its name and symbol, and the code
        object's VGPR / AGPR / SGPR counts, scratch bytes and spill counts (ur3e_amd/codeobj.py)."""
        e, l, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        name, sym = ctypes.create_string_buffer(160), ctypes.create_string_buffer(512)
        self._chk(self.L.ur3e_batch_tier_kernel(self.h, self.TIERS[tier] if isinstance(tier, str) else int(tier),
                                                ctypes.byref(e), ctypes.byref(l), ctypes.byref(r), name, 160, sym,
                                                512))
        out = {"envs_per_cu": e.value, "lds_bytes": l.value, "regs": r.value, "kernel": name.value.decode(),
               "symbol": sym.value.decode()}
        try:
            from .codeobj import resources
            res = resources(self.L._name, out["symbol"])
        except Exception as ex:  # llvm tools missing: the runtime figures above still stand
            res = {"error": repr(ex)}
        out["code_object"] = res
        return out

    def set_timing(self, on: bool = True):
        """Record HIP events around every (uncaptured) step, for last_step_ms()."""
        self._chk(self.L.ur3e_batch_set_timing(self.h, int(on)))

    def last_step_ms(self) -> float:
        ms = ctypes.c_float()
        self._chk(self.L.ur3e_batch_last_step_ms(self.h, ctypes.byref(ms)))
        return ms.value


__all__ = ["Batch", "make_config", "action_dim", "load_model", "load_library", "TASK_GYM_V2", "TASK_TRAJ_L", "TASK_MOVE_J",
           "TASK_CTRL", "TASK_GYM_V0", "TASK_IMIT_INDIRECT", "TASK_IMIT_DIRECT", "TASK_MOVE_L", "GAINS_L_MUG", "GAINS_V0",
           "GAINS_J", "GAINS_L_POS", "GAINS_L_ROT", "np"]
