"""Known-answer tests of the oracle's constraint physics that share no code with the kernel.

The GPU kernel is checked bit-for-bit against the oracle (tests/test_gpu_parity.py); these tests
check the oracle's contact, friction, equality and limit physics against answers derived here from
MuJoCo's documented soft-constraint model (MuJoCo 3.3.3 "Computation" chapter: solref/solimp
impedance, reference acceleration aref = -b v - k imp r, regulariser R = (1 - imp)/imp * A_hat,
elliptic friction cone with impratio), on small purpose-written MJCFs (tests/assets/kat_*.xml)
compiled by the model compiler.  Every expected value below is computed in this file with numpy
(the impedance sigmoid, the stiffness/damping constants, the steady-state equations), never by
calling the oracle's or the kernel's functions; the oracle only supplies the simulated state.

  1. box resting on a plane: total normal force = m g, tangential force 0, and the steady
     penetration solves the soft-contact equilibrium  D(r) K imp(r) (-r) = m g / 4 per corner;
  2. friction, elliptic cone, impratio 10: below mu m g the box creeps at the steady velocity the
     regularised friction rows imply, v = m g_x / (B sum_i D_t,i); above it slides with every
     cone on its surface, |f_t| = mu f_n, mu the pair's mixed friction (max of the geoms, or the
     priority geom's), and the momentum balance exact;
  3. connect equality: with A = A_hat (anchor at the centre of mass) the residual follows the
     critically damped recurrence of solref = (tc, 1): a = -(2/tc) v - r / tc^2, integrated by
     semi-implicit Euler, to rounding; and decays like (1 + t/tc) e^{-t/tc};
  4. joint limit: the row exists iff dist < margin, and a pendulum driven into its limit rests
     where D K imp (margin - dist) equals the gravity torque m g l cos q.
"""
import os

import numpy as np
import pytest
from scipy.optimize import brentq

HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(HERE, "assets")


def _model(name, gravity=None):
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    md = compile_mjcf(os.path.join(ASSETS, name + ".xml"))
    if gravity is not None:
        md["gravity"] = list(gravity)
    return md, to_ctypes(md)


def _data(mc):
    from oracle.pyoracle import OracleData
    return OracleData(mc)


# ---- MuJoCo's documented soft-constraint constants, restated independently -------------------
MINIMP, MAXIMP = 0.0001, 0.9999


def imp_of(solimp, r, margin=0.0):
    """impedance d(r) of solimp = (dmin, dmax, width, midpoint, power)"""
    dmin, dmax, width, mid, power = solimp
    dmin, dmax = np.clip(dmin, MINIMP, MAXIMP), np.clip(dmax, MINIMP, MAXIMP)
    if dmin == dmax:
        return dmin
    x = min(abs(r - margin) / width, 1.0)
    if x >= 1.0:
        return dmax
    if x <= mid:
        y = x ** power / mid ** (power - 1)
    else:
        y = 1.0 - (1.0 - x) ** power / (1.0 - mid) ** (power - 1)
    return dmin + y * (dmax - dmin)


def k_b(solref, solimp, dt):
    """stiffness K and damping B of aref = -B v - K imp r for a positive solref (timeconst, dampratio)"""
    tc, dr = max(solref[0], 2 * dt), solref[1]
    dmax = np.clip(solimp[1], MINIMP, MAXIMP)
    return 1.0 / (dmax ** 2 * tc ** 2 * dr ** 2), 2.0 / (dmax * tc)


def d_of(imp, a_hat):
    """D = 1/R with R = (1 - imp) / imp * A_hat"""
    return imp / ((1.0 - imp) * a_hat)


DEFAULT_SOLREF = (0.02, 1.0)
DEFAULT_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)
G = 9.81


def _settle(d, qpos, steps):
    d.set(qpos=qpos, qvel=np.zeros(d.nv))
    d.step(steps)
    return d.state(), d.contacts(), d.efc()


def test_box_rests_with_weight_and_penetration():
    md, mc = _model("kat_box_plane")
    m = 0.1
    st, con, efc = _settle(_data(mc), np.array(md["qpos0"], float)[:7], 3000)
    assert con["n"] == 4  # four corners of the bottom face
    fn = efc["force"][con["efc_address"]]
    ft = np.concatenate([efc["force"][con["efc_address"] + 1], efc["force"][con["efc_address"] + 2]])
    np.testing.assert_allclose(fn.sum(), m * G, rtol=1e-12)
    np.testing.assert_allclose(fn, m * G / 4, rtol=1e-9)
    assert np.abs(ft).max() < 1e-12
    assert np.abs(st["qvel"]).max() < 1e-12
    # steady penetration: per corner D(r) K imp(r) (-r) = m g / 4, A_hat = 1/m (free body, world plane)
    K, _ = k_b(DEFAULT_SOLREF, DEFAULT_SOLIMP, 0.001)

    def resid(r):
        imp = imp_of(DEFAULT_SOLIMP, r)
        return d_of(imp, 1.0 / m) * K * imp * (-r) - m * G / 4

    r_star = brentq(resid, -1e-3, -1e-9, xtol=1e-20, rtol=1e-15)
    np.testing.assert_allclose(con["dist"], r_star, rtol=1e-9)
    # the box centre sits r* below its contact-free height
    np.testing.assert_allclose(st["qpos"][2], 0.055111 + r_star, rtol=1e-12)


def _creep_or_slide(model, mass, gx, steps):
    """settle under vertical gravity, then continue the same state under gravity tilted by g_x"""
    md0, mc0 = _model(model)
    st0, _, _ = _settle(_data(mc0), np.array(md0["qpos0"], float)[:7], 1000)
    md, mc = _model(model, gravity=(gx, 0.0, -G))
    d = _data(mc)
    d.set(qpos=st0["qpos"], qvel=st0["qvel"])
    d.step(steps)
    return md, d.state(), d.contacts(), d.efc()


@pytest.mark.parametrize("model,mass", [("kat_box_plane", 0.1), ("kat_friction_mix", 0.5)])
def test_friction_stick_creep_velocity(model, mass):
    """below mu m g: every cone in its quadratic zone and the box creeps at v = m g_x / (B sum D_t)"""
    gx = 2.0
    md, st, con, efc = _creep_or_slide(model, mass, gx, 4000)
    assert con["n"] == 4
    a = con["efc_address"]
    assert (efc["state"][a] == 1).all()  # UR3O_STATE_QUADRATIC: inside the friction cone
    K, B = k_b(DEFAULT_SOLREF, DEFAULT_SOLIMP, 0.001)
    impratio = 10.0
    Dt = np.array([d_of(imp_of(DEFAULT_SOLIMP, r), 1.0 / mass) * impratio for r in con["dist"]])
    v_pred = mass * gx / (B * Dt.sum())
    np.testing.assert_allclose(st["qvel"][0], v_pred, rtol=1e-7)
    assert abs(st["qacc"][0]) < 1e-9 * gx
    # friction well below its cone bound
    fn, ft = efc["force"][a], efc["force"][a + 1]
    assert np.all(np.abs(ft) < con["friction"][:, 0] * fn)


@pytest.mark.parametrize("model,mass,mu", [("kat_friction_mix", 0.5, 0.6),  # equal priority: max(0.3, 0.6)
                                           ("kat_friction_priority", 0.5, 0.3)])  # plane has priority 1
def test_friction_slip_on_cone_surface(model, mass, mu):
    """above mu m g the box slides: every cone is on its surface, |f_t| = mu f_n with mu the pair's
    mixed friction, the friction opposes the slide, and the body's momentum balance
    m qacc = m g + sum_i frame_i' f_i holds exactly.  (Measured in the first steps of the slide:
    a fast-sliding soft elliptic contact pushes the box up and it chatters, so there is no clean
    sliding steady state to compare against.)"""
    gx = 7.0
    md, st, con, efc = _creep_or_slide(model, mass, gx, 4)
    assert con["n"] == 4
    np.testing.assert_array_equal(con["friction"][:, 0], mu)
    a = con["efc_address"]
    assert (efc["state"][a] == 4).all()  # UR3O_STATE_CONE: sliding
    fn = efc["force"][a]
    ftn = np.hypot(efc["force"][a + 1], efc["force"][a + 2])
    np.testing.assert_allclose(ftn, mu * fn, rtol=1e-10)
    F = np.zeros(3)
    for i in range(4):
        F += con["frame"][i].T @ efc["force"][a[i]:a[i] + 3]
    np.testing.assert_allclose(mass * st["qacc"][:3], mass * np.array([gx, 0.0, -G]) + F, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(-F[0], mu * fn.sum(), rtol=1e-9)  # all friction along -x
    assert st["qvel"][0] > 0 and abs(F[1]) < 1e-12 * mu * fn.sum()


def test_connect_residual_follows_solref():
    md, mc = _model("kat_connect")
    d = _data(mc)
    tc, h = 0.02, 0.001
    q = np.array(md["qpos0"], float)[:7]
    x0 = 0.01
    q[0] += x0  # the anchor (the box centre) starts 1 cm from its world point
    d.set(qpos=q, qvel=np.zeros(6))
    # independent discrete model: semi-implicit Euler of a = d aref = -(2/tc) v - x / tc^2
    x, v = x0, 0.0
    xs, xs_ref = [], []
    for n in range(300):
        d.step(1)
        a = -(2.0 / tc) * v - x / tc ** 2
        v = v + h * a
        x = x + h * v
        xs.append(d.state()["qpos"][0])
        xs_ref.append(x)
    xs, xs_ref = np.array(xs), np.array(xs_ref)
    np.testing.assert_allclose(xs, xs_ref, rtol=1e-9, atol=1e-15)
    st = d.state()
    assert np.abs(st["qpos"][1:3] - [0.0, 0.5]).max() < 1e-15  # no motion off the residual's axis
    # continuous-time check: critically damped decay (1 + t/tc) e^{-t/tc}, to O(h/tc)
    t = h * np.arange(1, 301)
    cont = x0 * (1 + t / tc) * np.exp(-t / tc)
    assert np.abs(xs - cont).max() < 0.05 * x0


def test_joint_limit_row_exists_within_margin():
    md, mc = _model("kat_hinge_limit")
    d = _data(mc)
    for q, rows in [(0.485, 0), (0.495, 1), (0.5, 1), (0.51, 1), (-0.485, 0), (-0.495, 1), (0.0, 0)]:
        d.set(qpos=np.array([q]), qvel=np.zeros(1))
        d.forward()
        e = d.efc()
        assert e["n"] == rows, (q, e["n"])
        if rows:
            side = 1 if q > 0 else -1
            np.testing.assert_allclose(e["pos"][0], side * (side * 0.5 - q), rtol=0, atol=1e-15)
            assert e["margin"][0] == 0.01 and e["J"][0, 0] == -side


def test_joint_limit_rest_position():
    md, mc = _model("kat_hinge_limit")
    d = _data(mc)
    st, _, efc = _settle(d, np.array([0.3]), 6000)
    m, l = 1.0, 0.2
    inertia = m * (0.02 ** 2 + 0.02 ** 2) / 3 + m * l ** 2  # box about its centre + parallel axis
    K, _ = k_b(DEFAULT_SOLREF, DEFAULT_SOLIMP, 0.001)
    margin = 0.01

    def resid(q):
        dist = 0.5 - q
        imp = imp_of(DEFAULT_SOLIMP, dist, margin)
        return d_of(imp, 1.0 / inertia) * K * imp * (margin - dist) - m * G * l * np.cos(q)

    q_star = brentq(resid, 0.49, 0.52, xtol=1e-16, rtol=1e-15)
    assert abs(st["qvel"][0]) < 1e-10
    np.testing.assert_allclose(st["qpos"][0], q_star, rtol=1e-10)
    np.testing.assert_allclose(efc["force"][0], m * G * l * np.cos(q_star), rtol=1e-8)
