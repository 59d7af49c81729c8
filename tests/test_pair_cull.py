"""The compact tier's pre-narrowphase cull (ur3e_amd/csrc/ur3e_wave.h: w_pair_apart), restated in numpy
and checked against the CPU oracle: over random gym ur3e-v2 states and states pressed against the table,
every candidate pair the cull removes has no contact in the oracle's contact list (so skipping its
narrowphase cannot change a result), and the cull removes most of the plane-box (and, on the mesh model,
plane-mesh) pairs that the bounding spheres keep.  The GPU side runs the same expressions; its bit-exactness is in the -m gpu parity tests."""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as po
from ur3e_amd import runtime as rt

PLANE, BOX, MESH = 0, 6, 7


def _apart(md, xp, xm, p):
    g1, g2 = md["cpair_geom1"][p], md["cpair_geom2"][p]
    t1, t2 = md["geom_type"][g1], md["geom_type"][g2]
    margin = md["cpair_margin"][p]
    if t1 == PLANE and t2 == MESH:
        pm = xm[g1]
        n = np.array([pm[2], pm[5], pm[8]])
        return n @ (xp[g2] - xp[g1]) - md["geom_rbound"][g2] > margin + 1e-9
    if t2 not in (BOX, MESH):
        return False
    size2 = np.asarray(md["geom_size"][g2])
    if t1 == PLANE:
        if t2 == MESH:
            return False
        pm, bm = xm[g1], xm[g2]
        n = np.array([pm[2], pm[5], pm[8]])
        dist = n @ (xp[g2] - xp[g1])
        ext = sum(size2[c] * abs(n[0] * bm[c] + n[1] * bm[3 + c] + n[2] * bm[6 + c]) for c in range(3))
        return dist - ext > margin + 1e-9
    if t1 not in (BOX, MESH):
        return False
    lim = margin + 1e-6 if MESH in (t1, t2) else margin  # a hull inside its geom_size box
    size1 = np.asarray(md["geom_size"][g1])
    a = np.asarray(xm[g1]).reshape(3, 3).T  # a[k] = column k
    b = np.asarray(xm[g2]).reshape(3, 3).T
    pp = xp[g2] - xp[g1]
    for ax in list(a) + list(b):
        ext = sum(size1[k] * abs(a[k] @ ax) for k in range(3)) + sum(size2[k] * abs(b[k] @ ax) for k in range(3))
        if abs(pp @ ax) - ext > lim:
            return True
    return False


def _states(md, mc):
    n = 32
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=2, max_episode_steps=60)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(1)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    low = np.array([0.29799994, 0.13349916, 0.0, 1.0])
    out = []
    for t in range(60):
        # every other window drives the gripper down onto the mug and table
        a = rng.uniform(lo, hi, size=(n, 4)) if (t // 15) % 2 == 0 else np.tile(low, (n, 1))
        ob.step(a)
        if t % 6 == 5:
            qp, qv, _, _ = ob.get_state()
            out.extend(zip(qp, qv))
    return out


@pytest.mark.parametrize("model", ["main", "main_mesh"])
def test_culled_pairs_have_no_oracle_contacts(model):
    md, mc = rt.load_model(model)
    L = po.lib()
    L.ur3o_data_geom_pose.argtypes = [ctypes.c_void_p] * 4
    ng = md["ngeom"]
    ncp = len(md["cpair_geom1"])
    plane_box = [p for p in range(ncp) if md["geom_type"][md["cpair_geom1"][p]] == PLANE
                 and md["geom_type"][md["cpair_geom2"][p]] in (BOX, MESH)]
    culled_pb = kept_pb = contacts_seen = 0
    for qp, qv in _states(md, mc):
        d = po.OracleData(mc, L=L)
        d.set(qpos=qp, qvel=qv)
        d.forward()
        xp, xm = np.zeros((ng, 3)), np.zeros((ng, 9))
        L.ur3o_data_geom_pose(ctypes.byref(mc), d.buf, xp.ctypes.data, xm.ctypes.data)
        touching = {tuple(sorted(g)) for g in d.contacts()["geoms"].tolist()}
        contacts_seen += len(touching)
        for p in range(ncp):
            if _apart(md, xp, xm, p):
                pair = tuple(sorted((md["cpair_geom1"][p], md["cpair_geom2"][p])))
                assert pair not in touching, f"pair {p} {pair} culled but in contact"
                culled_pb += p in plane_box
            else:
                kept_pb += p in plane_box
    assert contacts_seen > 0
    assert culled_pb > 5 * kept_pb, (culled_pb, kept_pb)


def test_mesh_hulls_inside_their_boxes_and_spheres():
    """the premise of the plane-mesh and mesh-pair clauses: every hull vertex of the mesh model lies in its
    geom's geom_size box and within its geom_rbound"""
    md, _ = rt.load_model("main_mesh")
    verts = np.asarray(md["mesh_vert"]).reshape(-1, 3)
    checked = 0
    for g in range(md["ngeom"]):
        if md["geom_type"][g] != MESH:
            continue
        i = md["geom_dataid"][g]
        v = verts[md["mesh_vertadr"][i]:md["mesh_vertadr"][i] + md["mesh_vertnum"][i]]
        assert (np.abs(v) <= np.asarray(md["geom_size"][g]) + 1e-15).all()
        assert (np.linalg.norm(v, axis=1) <= md["geom_rbound"][g] + 1e-12).all()
        checked += 1
    assert checked == 17
