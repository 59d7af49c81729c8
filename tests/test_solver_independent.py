"""The oracle's Newton constraint solve against an independent solver of the same problem.

The oracle (and bit-for-bit the kernel) solves MuJoCo's PRIMAL problem with Newton's method:
minimise over qacc  1/2 |qacc - qacc_smooth|_M^2 + s(J qacc - aref)  with s the regularised
constraint cost (quadratic rows, Huber friction loss, one-sided limits, and the three-zone elliptic
cone cost with mu = friction * sqrt(R_t / R_n)).  This test solves the DUAL problem the MuJoCo 3.3.3
documentation states for the same rows ("Computation: constraint model"):

    minimise over f in Omega   1/2 f' (A + R) f + f' (J qacc_smooth - aref),   A = J M^-1 J'
    Omega: equality rows free; friction-loss rows |f| <= frictionloss; limit rows f >= 0;
           contacts f_n >= |(f_1, f_2)| / friction  (the physical elliptic friction cone)

with an accelerated projected-gradient method (FISTA with adaptive restart, block-Jacobi scaled so
each cone stays a second-order cone) written here in numpy, then maps back
qacc = qacc_smooth + M^-1 J' f.  It shares nothing with the oracle's solver: not the cone zones, not
the Hessian, not the line search.  Agreement of qacc (and of the forces) to 1e-8 relative on
contact-rich main.xml states -- pad/box contacts sliding on their cones, saturated friction loss,
separating contacts -- pins that the primal cone cost and its mu scaling really are the dual of the
friction cone with the impratio regulariser.  Problem data (J, R, aref, M, qacc_smooth) come from
the oracle's own forward pass (oracle/ur3e_oracle_probe.c), which the kernel reproduces bit-exactly.
"""
import numpy as np
import pytest

TOL = 1e-8


def _solve_dual(e, con, st, iters=300000):
    J = e["J"]
    M = st["qM"]
    MiJt = np.linalg.solve(M, J.T)
    A = J @ MiJt
    R = e["R"]
    b = J @ st["qacc_smooth"] - e["aref"]
    nr = e["n"]
    s = np.ones(nr)
    cones = []
    for ci in range(con["n"]):
        a0 = con["efc_address"][ci]
        if a0 < 0:
            continue
        mu = con["friction"][ci, 0]
        s[a0 + 1] = s[a0 + 2] = 1.0 / mu  # g = s f maps the friction cone to |g_t| <= g_n
        cones.append(a0)
    cones = np.array(cones, int)
    Q0 = (A + np.diag(R)) * np.outer(1 / s, 1 / s)
    w = np.sqrt(np.diag(Q0)).copy()
    for a0 in cones:  # one scale per contact keeps the cone a cone
        w[a0:a0 + 3] = np.sqrt(np.mean(np.diag(Q0)[a0:a0 + 3]))
    s = s * w
    Si = 1.0 / s
    Q = (A + np.diag(R)) * np.outer(Si, Si)
    c = b * Si
    L = np.linalg.eigvalsh(Q).max()
    typ, fl = e["type"], e["frictionloss"]
    lim, fr = typ == 3, typ == 1

    def proj(g):
        g = g.copy()
        g[lim] = np.maximum(g[lim], 0)
        g[fr] = np.clip(g[fr], -fl[fr] * s[fr], fl[fr] * s[fr])
        if len(cones):
            gn = g[cones]
            gt = np.stack([g[cones + 1], g[cones + 2]], 1)
            tn = np.linalg.norm(gt, axis=1)
            inside, polar = tn <= gn, tn <= -gn
            alpha = (gn + tn) / 2
            g[cones] = np.where(inside, gn, np.where(polar, 0.0, alpha))
            sc = np.where(inside, 1.0, np.where(polar, 0.0, alpha / np.maximum(tn, 1e-300)))
            g[cones + 1] = gt[:, 0] * sc
            g[cones + 2] = gt[:, 1] * sc
        return g

    def obj(g):
        return 0.5 * g @ Q @ g + c @ g

    g = np.zeros(nr)
    y, t, fo = g.copy(), 1.0, 0.0
    for k in range(iters):
        gn = proj(y - (Q @ y + c) / L)
        tn = (1 + np.sqrt(1 + 4 * t * t)) / 2
        y = gn + (t - 1) / tn * (gn - g)
        fnew = obj(gn)
        if fnew > fo:  # adaptive restart
            y, tn = gn.copy(), 1.0
        if k > 100 and np.abs(gn - g).max() < 1e-17 * max(1.0, np.abs(gn).max()):
            g = gn
            break
        g, t, fo = gn, tn, fnew
    f = g * Si
    return f, st["qacc_smooth"] + MiJt @ f


def _contact_states(n_cone=3, n_other=3):
    """main.xml states from a grasp-region rollout of the oracle (gripper closing on the mug): the
    first n_cone with a sliding contact (a cone-surface row) and n_other with >= 5 contacts and none"""
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main")
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=3)
    n = 32
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(3)
    cone, other = [], []
    for step in range(600):
        a = np.zeros((n, 4))
        a[:, 0] = 0.29799994 + rng.normal(size=n) * 0.01
        a[:, 1] = 0.13349916 + rng.normal(size=n) * 0.01
        a[:, 2] = rng.uniform(0.02, 0.12, size=n)
        a[:, 3] = rng.uniform(0.5, 1.0, size=n)
        ob.step(a)
        if step % 40 != 39:
            continue
        qp, qv, wa, nc = ob.get_state()
        for i in np.flatnonzero(nc >= 4):
            d = po.OracleData(mc)
            d.set(qpos=qp[i], qvel=qv[i], ctrl=ob.diag(int(i))["ctrl"][:mc.nu], warm=wa[i])
            d.forward()
            if d.contacts()["n"] < 5:
                continue
            has_cone = bool((d.efc()["state"] == 4).any())
            (cone if has_cone else other).append(d)
        if len(cone) >= n_cone and len(other) >= n_other:
            break
    assert len(cone) >= n_cone and len(other) >= n_other
    return cone[:n_cone] + other[:n_other]


@pytest.fixture(scope="module")
def states():
    return _contact_states()


@pytest.mark.parametrize("k", range(6))
def test_newton_matches_independent_dual_solve(states, k):
    d = states[k]
    st, e, con = d.state(), d.efc(), d.contacts()
    assert con["n"] >= 5 and e["n"] > 3 * con["n"]  # contacts plus the equality / friction-loss rows
    f, qacc = _solve_dual(e, con, st)
    scale = max(1.0, np.abs(st["qacc"]).max())
    assert np.abs(qacc - st["qacc"]).max() <= TOL * scale, np.abs(qacc - st["qacc"]).max() / scale
    fscale = max(1.0, np.abs(e["force"]).max())
    assert np.abs(f - e["force"]).max() <= TOL * fscale
    # the physical cone holds for the oracle's forces: f_n >= |f_t| / friction (to rounding)
    for ci in range(con["n"]):
        a0 = con["efc_address"][ci]
        fn, ft = e["force"][a0], np.hypot(e["force"][a0 + 1], e["force"][a0 + 2])
        assert fn >= -1e-12 and ft <= con["friction"][ci, 0] * fn * (1 + 1e-9) + 1e-12
