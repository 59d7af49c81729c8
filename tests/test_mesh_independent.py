"""The convex narrowphase (ur3e_amd/csrc/convex.h: GJK + EPA, one contact per convex pair) pinned
independently of its source.  The oracle and the GPU both compile convex.h, so tests/test_gpu_mesh.py
only shows that the two compilations agree; here every contact the oracle reports for a convex pair of
tests/assets/mesh_scene.xml is re-derived with Qhull (scipy.spatial.ConvexHull) and numpy alone:

  * the Minkowski difference M = A - B of the two geoms' world vertices (hull vertices of a mesh, the 8
    corners of a box) is hulled; its facets are n_i . x <= c_i with unit outward n_i;
  * overlap (the origin inside M, every c_i > 0): the penetration depth is min_i c_i and the contact
    normal (from geom1 = A to geom2 = B) the n_i attaining it -- translating B by c_i n_i is the
    shortest move that separates them.  The oracle's dist must equal -depth and frame[0] that normal;
  * the contact point lies on the mid-plane of the two supporting planes along the normal
    (n . pos = (max_{a in A} n . a + min_{b in B} n . b) / 2), as the midpoint of the two witnesses;
  * separation (some c_i < 0): with zero margin there must be no contact for the pair.

Poses: random orientations of the free box mesh and hexagonal prism against the static box primitive,
the static tetrahedron mesh and each other, at random depths down to 1e-12 (where the sign of a
nearly-zero facet distance decides the normal's direction).  Geom world poses are composed here from
qpos and the compiled geom_pos / geom_quat (kinematics is pinned elsewhere); hull vertices come from
the compiled model (the hull itself is pinned against Qhull in tests/test_mesh.py)."""
import os

import numpy as np
import pytest

scipy_spatial = pytest.importorskip("scipy.spatial")

HERE = os.path.dirname(os.path.abspath(__file__))
SCENE = os.path.join(HERE, "assets", "mesh_scene.xml")
FAR = {"mbox": [-1.0, 1.0, 0.5], "prism": [1.0, 1.0, 0.5]}


def _quat_mat(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _rand_quat(rng):
    q = rng.normal(size=4)
    return q / np.linalg.norm(q)


@pytest.fixture(scope="module")
def scene():
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    md = compile_mjcf(SCENE)
    return md, to_ctypes(md)


def _local_verts(md, g):
    if md["geom_type"][g] == 7:  # mesh: the compiled hull vertices (mesh frame)
        k = md["geom_dataid"][g]
        a, n = md["mesh_vertadr"][k], md["mesh_vertnum"][k]
        return np.asarray(md["mesh_vert"], float)[a:a + n]
    assert md["geom_type"][g] == 6  # box
    h = np.asarray(md["geom_size"][g], float)
    return np.array([[sx * h[0], sy * h[1], sz * h[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])


def _world_verts(md, q, g):
    b = md["geom_bodyid"][g]
    gp, gR = np.asarray(md["geom_pos"][g], float), _quat_mat(md["geom_quat"][g])
    if b == 0:
        p, R = np.zeros(3), np.eye(3)
    else:
        name = md["body_names"][b]
        if name == "pusher":  # slide joint along x
            p = np.asarray(md["body_pos"][b], float) + np.array([q[md["jnt_qposadr"][2]], 0, 0])
            R = np.eye(3)
        else:
            a = md["jnt_qposadr"][b - 1]
            p, R = q[a:a + 3], _quat_mat(q[a + 3:a + 7])
    Rg = R @ gR
    pg = p + R @ gp
    return _local_verts(md, g) @ Rg.T + pg


def _mink(A, B):
    """facets (n_i unit outward, c_i) of hull(A - B)"""
    D = (A[:, None, :] - B[None, :, :]).reshape(-1, 3)
    h = scipy_spatial.ConvexHull(D)
    n, c = h.equations[:, :3], -h.equations[:, 3]
    return n, c


def _contacts(mc, q):
    from oracle.pyoracle import OracleData
    d = OracleData(mc)
    d.set(qpos=q, qvel=np.zeros(mc.nv))
    d.forward()
    return d.contacts()


def _check_pair(md, mc, q, ga, gb, stats):
    c = _contacts(mc, q)
    sel = [i for i in range(c["n"]) if set(c["geoms"][i]) == {ga, gb}]
    g1 = c["geoms"][sel[0]][0] if sel else ga
    g2 = gb if g1 == ga else ga
    A, B = _world_verts(md, q, g1), _world_verts(md, q, g2)
    n, cc = _mink(A, B)
    depth = cc.min()
    if depth < -1e-10:  # separated (margin 0): no contact
        assert not sel, f"contact reported for separated pair {ga},{gb} (gap {-depth:.3e})"
        stats["separated"] += 1
        return
    if depth < 1e-13:  # touching within rounding: either answer is right
        return
    assert len(sel) == 1, f"pair {ga},{gb} overlaps by {depth:.3e} but {len(sel)} contacts"
    i = sel[0]
    nrm = c["frame"][i][0]
    np.testing.assert_allclose(c["dist"][i], -depth, rtol=1e-7, atol=2e-10)
    # the normal: the minimising facet's (or, when facets tie within the EPA tolerance, one of them)
    ties = np.flatnonzero(cc <= depth + 2e-10)
    err = min(np.abs(nrm - n[t]).max() for t in ties)
    assert err < 1e-6, f"normal {nrm} vs {n[ties]} (depth {depth:.3e})"
    assert nrm @ n[ties[0]] > 0.99  # never reversed
    sA, sB = (A @ nrm).max(), (B @ nrm).min()
    np.testing.assert_allclose(c["pos"][i] @ nrm, 0.5 * (sA + sB), atol=1e-9)
    stats["overlap"] += 1
    stats["min_depth"] = min(stats["min_depth"], depth)


def _place(md, q, body, pos, quat):
    a = md["jnt_qposadr"][md["body_names"].index(body) - 1]
    q[a:a + 3] = pos
    q[a + 3:a + 7] = quat


def _base_q(md):
    q = np.array(md["qpos0"], float)
    for b, p in FAR.items():
        _place(md, q, b, p, [1, 0, 0, 0])
    q[md["jnt_qposadr"][2]] = -0.05  # pusher back
    return q


def _sink_to(md, q, body, g_other, pen, g_self):
    """translate `body` along z to where the two geoms just touch (bisection on the sign of the
    Minkowski hull's min facet offset, which is > 0 exactly when they overlap), then down by pen
    (a gap for pen < 0)"""
    a = md["jnt_qposadr"][md["body_names"].index(body) - 1]

    def overlap(z):
        q[a + 2] = z
        return _mink(_world_verts(md, q, g_self), _world_verts(md, q, g_other))[1].min() > 0
    hi = q[a + 2]
    lo = hi
    while not overlap(lo):
        lo -= 0.05
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        if overlap(mid):
            lo = mid
        else:
            hi = mid
    q[a + 2] = hi - pen


@pytest.mark.parametrize("other", ["block", "tetra", "prism"])
def test_epa_against_minkowski_hull(scene, other):
    md, mc = scene
    gn = md["geom_names"]
    gm, go = gn.index("mbox"), gn.index(other)
    rng = np.random.default_rng({"block": 1, "tetra": 2, "prism": 3}[other])
    stats = dict(overlap=0, separated=0, min_depth=np.inf)
    for k in range(60):
        q = _base_q(md)
        if other == "prism":
            _place(md, q, "prism", [0.3, 0.0, 0.1], _rand_quat(rng))
        # above the other geom's highest vertex, offset so that every feature pairing occurs
        top = _world_verts(md, q, go)
        x0 = top[top[:, 2].argmax()]
        _place(md, q, "mbox", [x0[0] + rng.uniform(-0.02, 0.02), x0[1] + rng.uniform(-0.02, 0.02), x0[2] + 0.2],
               _rand_quat(rng))
        # depths across scales, down to 1e-12, and a few small gaps
        pen = 10.0 ** rng.uniform(-12, -2.5) if k % 6 else -10.0 ** rng.uniform(-6, -3)
        _sink_to(md, q, "mbox", go, pen, gm)
        _check_pair(md, mc, q, gm, go, stats)
    assert stats["overlap"] >= 30 and stats["separated"] >= 3, stats
    print(other, stats)


def test_epa_normal_at_near_zero_depth(scene):
    """Face-on-face resting contact, the common case the EPA face orientation must get right: the box
    mesh flat on the box primitive (yaw only), penetrating by 1e-12 .. 1e-9.  The depth is the z overlap
    and the normal +z (from the block, geom1, to the mesh), never reversed."""
    md, mc = scene
    gn = md["geom_names"]
    gm, gbk = gn.index("mbox"), gn.index("block")
    rng = np.random.default_rng(11)
    body_q = np.array(md["geom_quat"][gm], float)  # the geom's frame permutes axes: undo it so faces align
    inv = np.array([body_q[0], -body_q[1], -body_q[2], -body_q[3]])
    for k in range(40):
        q = _base_q(md)
        yaw = rng.uniform(-np.pi, np.pi)
        qy = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
        # body quat = yaw * inverse(geom quat): the mesh's world frame is a pure yaw
        w1, v1 = qy[0], qy[1:]
        w2, v2 = inv[0], inv[1:]
        qb = np.r_[w1 * w2 - v1 @ v2, w1 * v2 + w2 * v1 + np.cross(v1, v2)]
        _place(md, q, "mbox", [0.1 + rng.uniform(-0.005, 0.005), rng.uniform(-0.005, 0.005), 0.3], qb)
        pen = 10.0 ** rng.uniform(-12, -9)
        a = md["jnt_qposadr"][md["body_names"].index("mbox") - 1]
        q[a + 2] += _world_verts(md, q, gbk)[:, 2].max() - _world_verts(md, q, gm)[:, 2].min() - pen
        depth = _world_verts(md, q, gbk)[:, 2].max() - _world_verts(md, q, gm)[:, 2].min()
        c = _contacts(mc, q)
        sel = [i for i in range(c["n"]) if set(c["geoms"][i]) == {gm, gbk}]
        assert len(sel) == 1, (k, depth)
        i = sel[0]
        assert c["geoms"][i][0] == gbk
        np.testing.assert_allclose(c["frame"][i][0], [0, 0, 1], atol=1e-9)
        np.testing.assert_allclose(c["dist"][i], -depth, rtol=1e-3, atol=1e-15)
