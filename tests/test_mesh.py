"""Real mesh support: mesh readers, convex hull, MuJoCo's mesh inertia and
inertial frame, and the convex narrowphase (ur3e_amd/csrc/convex.h, shared by the oracle and the GPU),
pinned on committed synthetic meshes (tests/assets/meshes/, tools/make_test_meshes.py) by closed forms:

  * a box written as a mesh has the box primitive's volume, centre and inertia; a unit tetrahedron has
    its closed-form inertia; a non-convex L prism's 'exact' volume is the L's, 'convex' overcounts it
    (the hull fills the notch) and 'legacy' never undercounts it;
  * the hull equals scipy's Qhull on random point clouds;
  * the box mesh on a plane gives the box primitive's four corner contacts (positions, normals, depths);
  * box-mesh against a box primitive (GJK/EPA, one contact) gives the separating-axis penetration depth
    and normal of the two boxes;
  * kat_mesh_box_plane.xml compiles to the inertia of kat_box_plane.xml and rests carrying m g with the
    same steady penetration (the box-primitive known answer of tests/test_physics_kat.py).
CPU only (the GPU is checked bit for bit against the oracle in tests/test_gpu_mesh.py)."""
import os

import numpy as np
import pytest

from ur3e_amd.model import mesh as M

HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(HERE, "assets")
MESHES = os.path.join(ASSETS, "meshes")
HALF = np.array([0.03, 0.02, 0.055111])


def _box_closed_form(h, rho=1.0):
    V = 8 * h[0] * h[1] * h[2]
    m = rho * V
    return V, m / 3 * np.array([h[1] ** 2 + h[2] ** 2, h[0] ** 2 + h[2] ** 2, h[0] ** 2 + h[1] ** 2])


def test_readers_stl_ascii_binary_obj(tmp_path):
    v, f = M.load_mesh(os.path.join(MESHES, "box.stl"))
    assert len(v) == 8 and len(f) == 12
    np.testing.assert_array_equal(np.sort(np.abs(v), axis=0)[0], HALF)
    v2, f2 = M.load_mesh(os.path.join(MESHES, "prism.stl"))  # binary
    assert len(v2) == 12 and len(f2) == 20
    v3, f3 = M.load_mesh(os.path.join(MESHES, "tetra.obj"), scale=(2.0, 2.0, 2.0))
    assert len(v3) == 4 and v3.max() == 2.0
    v4, f4 = M.load_mesh(os.path.join(MESHES, "lshape.obj"))  # quads and hexagons, fanned
    assert len(v4) == 12 and len(f4) == 2 * 4 + 6 * 2
    # round trip
    M.write_obj(str(tmp_path / "b.obj"), v, f)
    vb, fb = M.load_mesh(str(tmp_path / "b.obj"))
    np.testing.assert_array_equal(vb, v)


def test_hull_matches_qhull():
    from scipy.spatial import ConvexHull
    rng = np.random.default_rng(3)
    for n in (10, 60, 400):
        P = rng.normal(size=(n, 3)) * [1.0, 0.5, 2.0]
        idx, tri = M.convex_hull(P)
        h = ConvexHull(P)
        np.testing.assert_array_equal(idx, np.sort(h.vertices))
        vol, com, _ = M.mesh_inertia(P, tri, "exact")
        np.testing.assert_allclose(vol, h.volume, rtol=1e-12)
    with pytest.raises(ValueError):
        M.convex_hull(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0.0]]))  # flat


@pytest.mark.parametrize("mode", ["exact", "legacy", "convex"])
def test_box_mesh_inertia_equals_box(mode):
    v, f = M.load_mesh(os.path.join(MESHES, "box.stl"))
    vol, com, I = M.mesh_inertia(v, f, mode)
    V, Id = _box_closed_form(HALF)
    np.testing.assert_allclose(vol, V, rtol=1e-13)
    np.testing.assert_allclose(com, 0, atol=1e-17)
    np.testing.assert_allclose(I, np.diag(Id), rtol=1e-12, atol=1e-20)


def test_tetrahedron_inertia_closed_form():
    v, f = M.load_mesh(os.path.join(MESHES, "tetra.obj"))
    vol, com, I = M.mesh_inertia(v, f, "exact")
    np.testing.assert_allclose(vol, 1 / 6, rtol=1e-15)
    np.testing.assert_allclose(com, [0.25, 0.25, 0.25], rtol=1e-15)
    # unit right tetrahedron, density 1, about its centroid: I_ii = 1/80, I_ij = +1/480
    np.testing.assert_allclose(I, np.full((3, 3), 1 / 480) + np.eye(3) * (1 / 80 - 1 / 480), rtol=1e-12)


def test_nonconvex_legacy_overcounts():
    v, f = M.load_mesh(os.path.join(MESHES, "lshape.obj"))
    exact = M.mesh_inertia(v, f, "exact")[0]
    np.testing.assert_allclose(exact, 3 * 0.01 ** 3, rtol=1e-12)       # three unit squares x 1 cm
    assert M.mesh_inertia(v, f, "convex")[0] > exact                     # the hull fills the notch
    # legacy sums |tetrahedra| from the surface centroid: never less than the signed sum
    assert M.mesh_inertia(v, f, "legacy")[0] >= exact * (1 - 1e-12)


def test_legacy_reference_point_is_the_surface_centroid():
    """A mesh whose legacy volume depends on the reference point: a thin L prism whose long arm carries
    most of the surface.  The vertex mean and the surface centroid lie in different places, some
    tetrahedra change orientation between them, and the legacy volume is the sum of |tetrahedra| from
    the area-weighted face centroid (MuJoCo's legacy reference; parity vs MuJoCo unpinned), restated
    here with plain loops."""
    # L in the xy plane (long arm along x), extruded by h in z; non-convex at the notch
    P = [(0, 0), (10, 0), (10, 1), (1, 1), (1, 6), (0, 6)]
    h = 1.0
    v = np.array([(x, y, 0.0) for x, y in P] + [(x, y, h) for x, y in P])
    n = len(P)
    faces = []
    for i in range(n):  # side quads, outward for a counter-clockwise outline
        j = (i + 1) % n
        faces += [(i, j, n + j), (i, n + j, n + i)]
    for tri in ((0, 2, 1), (0, 3, 2), (0, 4, 3), (0, 5, 4)):  # bottom (fan from vertex 0), facing -z
        faces.append(tri)
        faces.append((n + tri[0], n + tri[2], n + tri[1]))  # top, facing +z
    f = np.array(faces)
    V_exact = M.mesh_inertia(v, f, "exact")[0]
    np.testing.assert_allclose(V_exact, (10 * 1 + 1 * 5) * h, rtol=1e-12)
    area, cen = [], []
    for a, b, c in f:
        area.append(0.5 * np.linalg.norm(np.cross(v[b] - v[a], v[c] - v[a])))
        cen.append((v[a] + v[b] + v[c]) / 3)
    ref = sum(A * C for A, C in zip(area, cen)) / sum(area)
    vol_from = lambda r: sum(abs(np.dot(v[a] - r, np.cross(v[b] - r, v[c] - r))) / 6 for a, b, c in f)
    assert abs(vol_from(ref) - vol_from(v.mean(axis=0))) > 1e-3  # the point matters for this mesh
    np.testing.assert_allclose(M.mesh_inertia(v, f, "legacy")[0], vol_from(ref), rtol=1e-12)


def _model(name):
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    md = compile_mjcf(os.path.join(ASSETS, name))
    return md, to_ctypes(md)


def test_mesh_body_compiles_to_box_inertia():
    mm, _ = _model("kat_mesh_box_plane.xml")
    mb, _ = _model("kat_box_plane.xml")
    assert mm["geom_type"][1] == 7 and mm["nmesh"] == 1 and mm["mesh_vertnum"][0] == 8
    np.testing.assert_allclose(mm["body_mass"], mb["body_mass"], rtol=1e-15)
    np.testing.assert_allclose(np.sort(mm["body_inertia"][1]), np.sort(mb["body_inertia"][1]), rtol=1e-12)
    np.testing.assert_allclose(mm["geom_rbound"][1], mb["geom_rbound"][1], rtol=1e-13)
    from ur3e_amd.model.compiler import compile_mjcf
    with pytest.raises(FileNotFoundError):
        compile_mjcf(os.path.join(ASSETS, "missing_mesh.xml"), meshes="mesh")
    # "auto" falls back to the documented box surrogate only for the reference's own mesh names
    with pytest.raises(KeyError):
        compile_mjcf(os.path.join(ASSETS, "missing_mesh.xml"))


def _contacts_at(mc, qpos):
    from oracle.pyoracle import OracleData
    d = OracleData(mc)
    d.set(qpos=qpos, qvel=np.zeros(mc.nv))
    d.forward()
    return d.contacts()


def _sorted(c):
    o = np.lexsort(np.round(c["pos"], 12).T[::-1])
    return c["pos"][o], c["frame"][o][:, 0], c["dist"][o]


def test_plane_mesh_contacts_equal_plane_box():
    _, mm = _model("kat_mesh_box_plane.xml")
    _, mb = _model("kat_box_plane.xml")
    rng = np.random.default_rng(1)
    for _ in range(20):
        q = np.zeros(7)
        q[:3] = [0.01, -0.02, 0.0551 - rng.uniform(0, 0.004)]
        ax = rng.normal(size=3) * 0.02
        ang = np.linalg.norm(ax)
        q[3:] = np.r_[np.cos(ang / 2), np.sin(ang / 2) * ax / ang]
        cm, cb = _contacts_at(mm, q), _contacts_at(mb, q)
        assert cm["n"] == cb["n"] and cm["n"] > 0
        for a, b in zip(_sorted(cm), _sorted(cb)):
            np.testing.assert_allclose(a, b, rtol=0, atol=1e-15)


def test_box_mesh_vs_box_epa_depth_equals_sat():
    """GJK/EPA on the box mesh against the static box primitive "block": the one contact's depth and
    normal equal the separating-axis answer for face-face overlaps (depth = the overlap along z)"""
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    md = compile_mjcf(os.path.join(ASSETS, "mesh_scene.xml"))
    mc = to_ctypes(md)
    names = md["body_names"]
    top = 0.02 + 0.02  # block: centre z 0.02, half height 0.02
    rng = np.random.default_rng(7)
    for k in range(10):
        pen = rng.uniform(1e-4, 3e-3)
        q = np.array(md["qpos0"], float)
        a_mbox = md["jnt_qposadr"][names.index("mbox") - 1]
        q[a_mbox:a_mbox + 7] = [0.1 + rng.uniform(-0.01, 0.01), rng.uniform(-0.01, 0.01),
                                top + 0.055111 - pen, 1, 0, 0, 0]
        a = md["jnt_qposadr"][md["joint_names"].index(md["joint_names"][1])]  # prism's free joint
        q[a:a + 7] = [-1.0, -1.0, 0.5, 1, 0, 0, 0]  # out of reach
        c = _contacts_at(mc, q)
        gm, gb = md["geom_names"].index("mbox"), md["geom_names"].index("block")
        sel = [i for i in range(c["n"]) if set(c["geoms"][i]) == {gm, gb}]
        assert len(sel) == 1  # one contact per convex pair (MuJoCo's default, no multiccd)
        i = sel[0]
        np.testing.assert_allclose(c["dist"][i], -pen, rtol=1e-9, atol=1e-13)
        assert c["geoms"][i][0] == gb  # geom1 = the box (lower type), normal from it to the mesh: +z
        np.testing.assert_allclose(c["frame"][i][0], [0, 0, 1], atol=1e-9)


def test_mesh_box_rests_like_box_primitive():
    from oracle.pyoracle import OracleData
    mm, cm = _model("kat_mesh_box_plane.xml")
    mb, cb = _model("kat_box_plane.xml")
    out = []
    for md, mc in ((mm, cm), (mb, cb)):
        d = OracleData(mc)
        d.set(qpos=np.array(md["qpos0"], float)[:7], qvel=np.zeros(6))
        d.step(3000)
        st, con, efc = d.state(), d.contacts(), d.efc()
        out.append((st, con, efc))
    (sm, cmn, em), (sb, cbn, eb) = out
    assert cmn["n"] == 4 == cbn["n"]
    fm = em["force"][cmn["efc_address"]]
    np.testing.assert_allclose(fm.sum(), 0.1 * 9.81, rtol=1e-12)
    np.testing.assert_allclose(np.sort(cmn["dist"]), np.sort(cbn["dist"]), rtol=1e-9)
    np.testing.assert_allclose(sm["qpos"][:3], sb["qpos"][:3], atol=1e-12)
