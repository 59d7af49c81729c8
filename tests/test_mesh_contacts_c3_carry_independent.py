"""The mesh contact geometry in the scripted pick's carry regime, pinned independently of convex.h.

convex.h (GJK + EPA) is one source compiled into the oracle and into every GPU tier, so GPU-vs-oracle parity
cannot catch a defect in it.  tests/test_mesh_contacts_main_independent.py checks contact existence and depth
of main_mesh pairs on holding poses; this test follows the move_l_mug scripted pick on main_mesh
(controller/move_l_mug.py:67-81, one mj_step per build_traj_l_pick_place row) through the grasp, the lift and
the carry (rows 1,800-4,200: the closed fingers' linkage meshes touch each other and the mug, so EPA runs
every row), and re-derives every box-mesh and mesh-mesh contact the oracle reports with Qhull and numpy alone:

  * the Minkowski difference M = A - B of the two geoms' world vertices (hull vertices of a mesh, the corners
    of a box) is hulled; facets n_i . x <= c_i with unit outward n_i;
  * overlap (every c_i > 0): exactly one contact, dist = -(min_i c_i) (EPA's tolerance), its normal
    frame[0] (geom1 -> geom2) the n_i attaining the minimum (any facet within the tolerance of it when
    facets tie), never reversed, and its position on the mid-plane of the two supporting planes along that
    normal (the midpoint of EPA's witness points);
  * separation by more than 1e-9 (margin 0): no contact for the pair.

World poses come from the compiler's own numpy kinematics (ur3e_amd/model/compiler.py _fk), not the oracle's.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
scipy_spatial = pytest.importorskip("scipy.spatial")

ROWS = (1800, 4200, 150)  # the carry regime, every 150th row


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


def test_c3_carry_mesh_contacts_against_minkowski_hull():
    from helpers import oracle_pick_place_rows
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    from ur3e_amd.model.compiler import _fk
    md, mc = rt.load_model("main_mesh")
    gt = np.asarray(md["geom_type"])
    gn = md["geom_names"]
    cfg = rt.make_config(task=rt.TASK_TRAJ_L, frame_skip=1, max_episode_steps=0, auto_reset=False, reset_noise=3,
                         reset_key=md["id_key_down"], model=md, seed=0)
    n = 4
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rows = oracle_pick_place_rows(md, mc, ob)
    # box-mesh and mesh-mesh candidate pairs (plane-mesh has its own vertex rule, pinned in test_mesh.py)
    pairs = {(int(md["cpair_geom1"][p]), int(md["cpair_geom2"][p])) for p in range(md["ncpair"])
             if 7 in (gt[md["cpair_geom1"][p]], gt[md["cpair_geom2"][p]])
             and 0 not in (gt[md["cpair_geom1"][p]], gt[md["cpair_geom2"][p]])}
    r0, r1, every = ROWS
    stats = dict(states=0, overlap=0, apart=0, mesh_mesh_overlap=0, ties=0, max_depth=0.0, max_normal_err=0.0,
                 max_mid_err=0.0)
    kinds = set()
    for t in range(r1):
        ob.step(rows[:, t])
        if t < r0 or (t - r0) % every:
            continue
        qp, qv, _, _ = ob.get_state()
        for i in range(n):
            d = po.OracleData(mc)
            d.set(qpos=qp[i], qvel=qv[i])
            d.forward()
            c = d.contacts()
            xpos, xmat, _, _, _ = _fk(md, qp[i])
            stats["states"] += 1
            for ga, gb in pairs:
                sel = [k for k in range(c["n"]) if {int(c["geoms"][k][0]), int(c["geoms"][k][1])} == {ga, gb}]
                g1 = int(c["geoms"][sel[0]][0]) if sel else ga
                g2 = gb if g1 == ga else ga
                A, B = _world(md, xpos, xmat, g1), _world(md, xpos, xmat, g2)
                ra = np.linalg.norm(A - A.mean(0), axis=1).max()
                rb = np.linalg.norm(B - B.mean(0), axis=1).max()
                if np.linalg.norm(A.mean(0) - B.mean(0)) > ra + rb + 1e-6:
                    assert not sel, (t, i, gn[ga], gn[gb])
                    continue
                D = (A[:, None, :] - B[None, :, :]).reshape(-1, 3)
                h = scipy_spatial.ConvexHull(D)
                nrm_f, cc = h.equations[:, :3], -h.equations[:, 3]
                depth = cc.min()
                where = f"row {t} env {i} {gn[g1]}-{gn[g2]}"
                if depth < -1e-9:
                    assert not sel, f"{where}: contact for a pair apart by {-depth:.3e}"
                    stats["apart"] += 1
                    continue
                if depth < 1e-9:
                    continue  # touching within rounding: either answer is right
                assert len(sel) == 1, f"{where}: overlap {depth:.3e} but {len(sel)} contacts"
                k = sel[0]
                # EPA stops within its tolerance of the polytope's closest face (convex.h), relative to depth
                np.testing.assert_allclose(c["dist"][k], -depth, rtol=1e-6, atol=1e-9, err_msg=where)
                nrm = np.asarray(c["frame"][k][0], float)
                ties = np.flatnonzero(cc <= depth + max(1e-9, 1e-6 * depth))
                stats["ties"] += len(ties) > 1
                err = min(np.abs(nrm - nrm_f[j]).max() for j in ties)
                assert err < 1e-5, f"{where}: normal {nrm} vs {nrm_f[ties]} (depth {depth:.3e})"
                assert nrm @ nrm_f[ties[0]] > 0.99, f"{where}: normal reversed"
                sA, sB = (A @ nrm).max(), (B @ nrm).min()
                mid = abs(c["pos"][k] @ nrm - 0.5 * (sA + sB))
                assert mid < 1e-8, f"{where}: contact {mid:.3e} off the mid-plane"
                stats["overlap"] += 1
                both_mesh = gt[g1] == 7 and gt[g2] == 7
                stats["mesh_mesh_overlap"] += int(both_mesh)
                kinds.add("mesh-mesh" if both_mesh else "box-mesh")
                stats["max_depth"] = max(stats["max_depth"], depth)
                stats["max_normal_err"] = max(stats["max_normal_err"], err)
                stats["max_mid_err"] = max(stats["max_mid_err"], mid)
    print(stats, kinds)
    # the carry regime does exercise EPA on mesh pairs, mesh-mesh included, and separations are checked too
    assert stats["overlap"] >= 20 and stats["mesh_mesh_overlap"] >= 10 and stats["apart"] >= 20, stats
