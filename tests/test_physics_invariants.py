"""Physics known-answer and invariant tests of the CPU oracle (test infrastructure; the GPU path is
bit-identical to it, tests/test_gpu_parity.py).  MuJoCo itself is absent, so these pin the oracle's
restatement of mj_step on facts that hold for any correct rigid-body engine with MuJoCo's
integrator, independent of this implementation:

- free fall of the unconstrained mug under semi-implicit Euler: v_n = -n h g, z_n = z_0 - h^2 g n(n+1)/2,
  orientation and horizontal position unchanged (mj_Euler, free joint, no contacts);
- RNE bias is affine-plus-quadratic in the velocity: b(q, 2v) - b(q, 0) = 4 (b(q, v) - b(q, 0));
- passivity of the Lagrangian form: v' C(q, v) v = 1/2 v' dM/dt v, with C v = b(q, v) - b(q, 0) and
  dM/dt along v from central differences of the CRB mass matrix (checks CRB against RNE);
- the mass matrix is symmetric positive definite.
"""
import numpy as np
import pytest

from oracle import pyoracle as po
from ur3e_amd import runtime as rt


@pytest.fixture(scope="module")
def main_model():
    return rt.load_model("main")


def _hinge_qadr(md):
    """(qpos address, dof address) of every hinge/slide joint"""
    out = []
    for j in range(md["njnt"]):
        if md["jnt_type"][j] != 0:  # not free
            out.append((md["jnt_qposadr"][j], md["jnt_dofadr"][j]))
    return out


def _free_joint(md):
    for j in range(md["njnt"]):
        if md["jnt_type"][j] == 0:
            return md["jnt_qposadr"][j], md["jnt_dofadr"][j]
    raise AssertionError("main.xml has the mug's free joint")


def test_mug_free_fall_exact(main_model):
    md, mc = main_model
    qa, da = _free_joint(md)
    assert all(md["dof_damping"][da + k] == 0 for k in range(6))
    cfg = rt.make_config(task=rt.TASK_CTRL, frame_skip=1, max_episode_steps=0, auto_reset=False,
                         reset_noise=False, reset_key=md["id_key_down"], model=md, seed=0)
    ob = po.OracleBatch(mc, po.config_from(cfg), 1)
    q = np.array(md["key_qpos"][md["id_key_down"]], dtype=np.float64)
    q[qa:qa + 3] = [2.0, 2.0, 1.0]  # far from the robot and the table: no contacts
    q[qa + 3:qa + 7] = [0.9238795325112867, 0.0, 0.3826834323650898, 0.0]
    ob.set_state(q[None], np.zeros((1, md["nv"])))
    h, g = md["timestep"], -md["gravity"][2]
    n = 150
    for _ in range(n):
        ob.step(np.zeros((1, md["nu"])))
    qp, qv, _, nc = ob.get_state()
    assert nc[0] == 0
    np.testing.assert_allclose(qv[0, da:da + 3], [0.0, 0.0, -n * h * g], rtol=0, atol=1e-9)
    np.testing.assert_allclose(qv[0, da + 3:da + 6], 0.0, atol=1e-12)
    np.testing.assert_allclose(qp[0, qa:qa + 3], [2.0, 2.0, 1.0 - h * h * g * n * (n + 1) / 2], rtol=0, atol=1e-9)
    np.testing.assert_allclose(qp[0, qa + 3:qa + 7], q[qa + 3:qa + 7], atol=1e-12)


def _state(md, rng):
    q = np.array(md["key_qpos"][md["id_key_down"]], dtype=np.float64)
    for qa, _ in _hinge_qadr(md):
        q[qa] += rng.uniform(-0.3, 0.3)
    v = np.zeros(md["nv"])
    for _, da in _hinge_qadr(md):
        v[da] = rng.uniform(-1.0, 1.0)
    return q, v


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_bias_quadratic_in_velocity(main_model, seed):
    md, mc = main_model
    q, v = _state(md, np.random.default_rng(seed))
    b0 = po.forward_state(mc, q, np.zeros_like(v))["qfrc_bias"]
    b1 = po.forward_state(mc, q, v)["qfrc_bias"]
    b2 = po.forward_state(mc, q, 2 * v)["qfrc_bias"]
    np.testing.assert_allclose(b2 - b0, 4 * (b1 - b0), rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_passivity_crb_vs_rne(main_model, seed):
    md, mc = main_model
    q, v = _state(md, np.random.default_rng(10 + seed))
    M = po.forward_state(mc, q, np.zeros_like(v))["qM"]
    np.testing.assert_allclose(M, M.T, rtol=0, atol=1e-15)
    assert np.linalg.eigvalsh(M).min() > 0
    cv = po.forward_state(mc, q, v)["qfrc_bias"] - po.forward_state(mc, q, np.zeros_like(v))["qfrc_bias"]
    eps = 1e-6
    dq = np.zeros_like(q)
    for qa, da in _hinge_qadr(md):
        dq[qa] = v[da]
    Mp = po.forward_state(mc, q + eps * dq)["qM"]
    Mm = po.forward_state(mc, q - eps * dq)["qM"]
    mdot = (Mp - Mm) / (2 * eps)
    lhs, rhs = v @ cv, 0.5 * v @ mdot @ v
    assert abs(lhs - rhs) <= 1e-6 * max(1.0, abs(rhs)), (lhs, rhs)
