"""main.xml with its convex stand-in meshes: every box-mesh and mesh-mesh pair the oracle settles, checked
against Qhull and numpy alone (independent of convex.h, as tests/test_mesh_independent.py does for a
synthetic scene).  States: the gripper's linkage meshes resting on the mug and a pad box on the upper-arm mesh
(the holding poses of tests/test_gpu_mesh_main.py), every one of 12 move_j steps of 32 envs (the pre-fix GJK
gave a spurious contact at step 11 of env 10).  For every candidate pair with a mesh
whose Minkowski difference (world hull vertices; boxes by their corners) is hulled by Qhull:

  * the origin outside the hull by more than 1e-9 (the pair apart, margin 0): no contact may be reported.
    Round 5 found the old GJK reporting overlap here for nearly flat simplices, after which EPA returned a
    "contact" at positive distance; convex.h's separating-axis exit removed those;
  * the origin inside by more than 1e-9: exactly one contact, at -(penetration depth) = -(the smallest facet
    offset), within EPA's tolerance.

World poses come from the compiler's own numpy kinematics (ur3e_amd/model/compiler.py _fk), not the
oracle's."""
import numpy as np
import pytest

scipy_spatial = pytest.importorskip("scipy.spatial")


def _q2mat(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _local_verts(md, g):
    if md["geom_type"][g] == 7:
        k = md["geom_dataid"][g]
        a, n = md["mesh_vertadr"][k], md["mesh_vertnum"][k]
        return np.asarray(md["mesh_vert"], float)[a:a + n]
    h = np.asarray(md["geom_size"][g], float)
    return np.array([[sx * h[0], sy * h[1], sz * h[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])


def _world(md, xpos, xmat, g):
    b = md["geom_bodyid"][g]
    R = xmat[b] @ _q2mat(md["geom_quat"][g])
    p = xpos[b] + xmat[b] @ np.asarray(md["geom_pos"][g], float)
    return _local_verts(md, g) @ R.T + p


def test_main_mesh_pairs_against_qhull():
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    from ur3e_amd.model.compiler import _fk
    md, mc = rt.load_model("main_mesh")
    gt = np.asarray(md["geom_type"])
    n, steps = 32, 12
    cfg = rt.make_config(task=rt.TASK_MOVE_J, frame_skip=1, model=md, seed=4, reset_noise=False,
                         reset_key=md["id_key_down"], max_episode_steps=0, auto_reset=False)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(9)
    q = np.tile(np.array(md["key_qpos"][md["id_key_down"]], float), (n, 1))
    half = n // 2
    q[:half, 1] += rng.uniform(0.36, 0.44, size=half)   # the gripper's linkage meshes on the mug
    q[half:, 3] += rng.uniform(1.15, 1.25, size=n - half)  # a pad box on the upper-arm mesh
    ob.set_state(q, np.zeros((n, md["nv"])))
    target = np.concatenate([q[:, :6], np.zeros((n, 1))], axis=1)
    pairs = [(md["cpair_geom1"][p], md["cpair_geom2"][p]) for p in range(md["ncpair"])
             if gt[md["cpair_geom2"][p]] == 7 and gt[md["cpair_geom1"][p]] != 0]
    stats = dict(apart=0, overlap=0, states=0)
    for t in range(steps):
        ob.step(target)
        qp, qv, _, _ = ob.get_state()
        for i in range(n):
            d = po.OracleData(mc)
            d.set(qpos=qp[i], qvel=qv[i])
            d.forward()
            c = d.contacts()
            xpos, xmat, _, _, _ = _fk(md, qp[i])
            stats["states"] += 1
            for g1, g2 in pairs:
                A, B = _world(md, xpos, xmat, g1), _world(md, xpos, xmat, g2)
                # bounding spheres first (most pairs are far apart)
                ra = np.linalg.norm(A - A.mean(0), axis=1).max()
                rb = np.linalg.norm(B - B.mean(0), axis=1).max()
                if np.linalg.norm(A.mean(0) - B.mean(0)) > ra + rb + 1e-6:
                    continue
                sel = [k for k in range(c["n"]) if (c["geoms"][k][0], c["geoms"][k][1]) == (g1, g2)]
                if not sel and t % 4 != 3:
                    continue  # pairs without a contact: every fourth step (a missed contact would persist)
                D = (A[:, None, :] - B[None, :, :]).reshape(-1, 3)
                h = scipy_spatial.ConvexHull(D)
                off = -h.equations[:, 3]  # > 0: the origin inside that facet's half-space
                depth = off.min()
                if depth < -1e-9:
                    assert not sel, (f"state {t}/{i}: contact for apart pair {md['geom_names'][g1]}, "
                                     f"{md['geom_names'][g2]} (gap >= {-depth:.3e}, dist {c['dist'][sel[0]]:.3e})")
                    stats["apart"] += 1
                elif depth > 1e-9:
                    assert len(sel) == 1, f"state {t}/{i}: pair {g1},{g2} overlaps by {depth:.3e}, {len(sel)} contacts"
                    np.testing.assert_allclose(c["dist"][sel[0]], -depth, rtol=1e-6, atol=1e-9)
                    stats["overlap"] += 1
    print(stats)
    assert stats["overlap"] > 0 and stats["apart"] > 0
