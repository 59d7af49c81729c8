"""Mesh assets for the model compiler: STL/OBJ readers, the convex hull, and MuJoCo's mesh inertia.

The reference MJCF (assets/main.xml:16-42) declares STL/OBJ meshes that the reference repository does
not ship (.gitignore:2-4).  When the files are present (a user who has them), the compiler builds the
model with real mesh geoms through this module instead of the box surrogate (surrogate.py):

* readers: binary and ASCII STL, Wavefront OBJ (v / f records, polygons fanned into triangles), with
  the MJCF `scale` applied to the vertices (mjCMesh);
* `convex_hull`: incremental 3-D hull (the hull is what MuJoCo collides with: `mjCMesh` builds it with
  qhull; here a deterministic incremental construction, cross-checked against scipy's Qhull in
  tests/test_mesh.py);
* `mesh_inertia`: volume, centre of mass and inertia of the solid, by signed tetrahedra from a
  reference point (Mirtich's covariance formula per tetrahedron).  MuJoCo's `<mesh inertia=...>`
  modes: "convex" (the hull), "exact" (the closed mesh, signed volumes), "legacy" (MuJoCo's default in
  3.3.3: tetrahedra from the vertex centroid with absolute volumes; equal to the others for convex
  meshes), "shell" (mass on the surface, area-weighted triangles);
* `principal_frame`: MuJoCo re-expresses every mesh in its inertial frame (centre of mass at the
  origin, principal axes as the coordinate axes; the geom's pos/quat absorb the offset), which is
  what the model image stores.
"""
from __future__ import annotations

import os
import struct

import numpy as np


# --------------------------------------------------------------------------------------------
# readers
def read_stl(path: str):
    """(vertices [n, 3], faces [m, 3]) of an STL file (binary or ASCII); vertices are merged exactly."""
    with open(path, "rb") as f:
        data = f.read()
    tris = None
    if len(data) >= 84:
        n = struct.unpack_from("<I", data, 80)[0]
        if 84 + 50 * n == len(data):
            rec = np.frombuffer(data, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                                count=n, offset=84)
            tris = rec["v"].astype(np.float64)
    if tris is None:
        txt = data.decode("ascii", errors="replace").split()
        vs = []
        i = 0
        while i < len(txt):
            if txt[i] == "vertex":
                vs.append([float(txt[i + 1]), float(txt[i + 2]), float(txt[i + 3])])
                i += 4
            else:
                i += 1
        if len(vs) % 3:
            raise ValueError(f"{path}: malformed ASCII STL")
        tris = np.asarray(vs, dtype=np.float64).reshape(-1, 3, 3)
    return _merge(tris)


def read_obj(path: str):
    """(vertices, faces) of a Wavefront OBJ file: `v x y z` and `f a b c ...` (1-based, v/vt/vn forms,
    negative indices), polygons fanned from their first vertex."""
    vs, fs = [], []
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                vs.append([float(p[1]), float(p[2]), float(p[3])])
            elif p[0] == "f":
                idx = []
                for tok in p[1:]:
                    k = int(tok.split("/")[0])
                    idx.append(k - 1 if k > 0 else len(vs) + k)
                for j in range(1, len(idx) - 1):
                    fs.append([idx[0], idx[j], idx[j + 1]])
    return np.asarray(vs, dtype=np.float64).reshape(-1, 3), np.asarray(fs, dtype=np.int64).reshape(-1, 3)


def _merge(tris):
    v = tris.reshape(-1, 3)
    uniq, inv = np.unique(v, axis=0, return_inverse=True)
    return uniq, inv.reshape(-1, 3).astype(np.int64)


def load_mesh(path: str, scale=(1.0, 1.0, 1.0)):
    ext = os.path.splitext(path)[1].lower()
    if ext == ".stl":
        v, f = read_stl(path)
    elif ext == ".obj":
        v, f = read_obj(path)
    else:
        raise ValueError(f"unsupported mesh format: {path}")
    return v * np.asarray(scale, dtype=np.float64), f


def write_stl_ascii(path: str, v, f):
    """test helper / tooling: an ASCII STL of the triangles f over vertices v"""
    with open(path, "w") as out:
        out.write("solid ur3e\n")
        for t in f:
            a, b, c = v[t[0]], v[t[1]], v[t[2]]
            n = np.cross(b - a, c - a)
            ln = np.linalg.norm(n)
            n = n / ln if ln > 0 else n
            out.write(f"facet normal {n[0]:.17g} {n[1]:.17g} {n[2]:.17g}\n outer loop\n")
            for p in (a, b, c):
                out.write(f"  vertex {p[0]:.17g} {p[1]:.17g} {p[2]:.17g}\n")
            out.write(" endloop\nendfacet\n")
        out.write("endsolid ur3e\n")


def write_obj(path: str, v, f):
    with open(path, "w") as out:
        for p in v:
            out.write(f"v {p[0]:.17g} {p[1]:.17g} {p[2]:.17g}\n")
        for t in f:
            out.write(f"f {t[0] + 1} {t[1] + 1} {t[2] + 1}\n")


# --------------------------------------------------------------------------------------------
# convex hull
def convex_hull(v, eps: float | None = None):
    """Incremental 3-D convex hull.  Returns (hull vertex indices into v, ascending; triangles over those
    indices with outward orientation).  Raises on degenerate (flat) input."""
    v = np.asarray(v, dtype=np.float64)
    n = len(v)
    if n < 4:
        raise ValueError("convex hull needs at least 4 points")
    ext = float(np.max(np.ptp(v, axis=0)))
    eps = 1e-10 * max(ext, 1e-300) if eps is None else eps
    # initial tetrahedron: extreme x, farthest from that line, farthest from that plane
    i0 = int(np.argmin(v[:, 0]))
    i1 = int(np.argmax(np.linalg.norm(v - v[i0], axis=1)))
    d = v[i1] - v[i0]
    cr = np.linalg.norm(np.cross(v - v[i0], d), axis=1)
    i2 = int(np.argmax(cr))
    nrm = np.cross(v[i1] - v[i0], v[i2] - v[i0])
    if np.linalg.norm(nrm) <= eps * ext:
        raise ValueError("degenerate point set (collinear)")
    pd = (v - v[i0]) @ nrm
    i3 = int(np.argmax(np.abs(pd)))
    if abs(pd[i3]) <= eps * np.linalg.norm(nrm):
        raise ValueError("degenerate point set (flat)")
    cen = (v[i0] + v[i1] + v[i2] + v[i3]) / 4.0
    faces = []

    def add(a, b, c):
        fn = np.cross(v[b] - v[a], v[c] - v[a])
        if np.dot(fn, v[a] - cen) < 0:
            b, c = c, b
            fn = -fn
        ln = np.linalg.norm(fn)
        faces.append([a, b, c, fn / ln, float(np.dot(fn / ln, v[a]))])

    for a, b, c in ((i0, i1, i2), (i0, i1, i3), (i0, i2, i3), (i1, i2, i3)):
        add(a, b, c)
    done = {i0, i1, i2, i3}
    for p in range(n):
        if p in done:
            continue
        vis = [k for k, f in enumerate(faces) if np.dot(f[3], v[p]) - f[4] > eps]
        if not vis:
            continue
        edges = {}
        for k in vis:
            a, b, c = faces[k][:3]
            for e in ((a, b), (b, c), (c, a)):
                if (e[1], e[0]) in edges:
                    del edges[(e[1], e[0])]
                else:
                    edges[e] = True
        vs = set(vis)
        faces = [f for k, f in enumerate(faces) if k not in vs]
        for (a, b) in edges:
            fn = np.cross(v[b] - v[a], v[p] - v[a])
            ln = np.linalg.norm(fn)
            if ln <= 0:
                continue
            faces.append([a, b, p, fn / ln, float(np.dot(fn / ln, v[a]))])
    idx = sorted({int(x) for f in faces for x in f[:3]})
    tri = np.asarray([[f[0], f[1], f[2]] for f in faces], dtype=np.int64)
    return np.asarray(idx, dtype=np.int64), tri


# --------------------------------------------------------------------------------------------
# mass properties
def _tet_props(a, b, c):
    """signed volume and second-moment covariance of tetrahedron (0, a, b, c) (rows of [k, 3] arrays)"""
    vol = np.einsum("ij,ij->i", a, np.cross(b, c)) / 6.0
    s = a + b + c
    cov = (np.einsum("i,ij,ik->ijk", vol, a, a) + np.einsum("i,ij,ik->ijk", vol, b, b) +
           np.einsum("i,ij,ik->ijk", vol, c, c) + np.einsum("i,ij,ik->ijk", vol, s, s)) / 20.0
    return vol, s / 4.0, cov


def mesh_inertia(v, f, mode: str = "legacy"):
    """(volume, com [3], inertia tensor about the com [3, 3]) of the solid bounded by triangles f over v
    (unit density).  mode: 'exact' (signed tetrahedra from the origin), 'convex' (the same over the convex
    hull), 'legacy' (tetrahedra from the area-weighted surface centroid, absolute volumes), 'shell' (unit surface
    density: triangle areas at their centroids with the thin-triangle second moments)."""
    v = np.asarray(v, dtype=np.float64)
    f = np.asarray(f, dtype=np.int64)
    if mode == "convex":
        hv, hf = convex_hull(v)
        return mesh_inertia(v, hf, "exact")
    if mode == "shell":
        a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
        area = 0.5 * np.linalg.norm(np.cross(b - a, c - a), axis=1)
        A = area.sum()
        com = (area[:, None] * (a + b + c) / 3.0).sum(0) / A
        a, b, c = a - com, b - com, c - com
        s = a + b + c
        cov = np.zeros((3, 3))
        for k in range(len(f)):  # second moment of a triangle: A/12 (sum v v^T + s s^T)
            cov += area[k] / 12.0 * (np.outer(a[k], a[k]) + np.outer(b[k], b[k]) + np.outer(c[k], c[k]) +
                                     np.outer(s[k], s[k]))
        return A, com, np.trace(cov) * np.eye(3) - cov
    if mode == "legacy":
        # MuJoCo's legacy volume: tetrahedra from the surface centroid (face centroids weighted by face
        # area), absolute volumes.  For a convex or star-shaped mesh any interior point gives the same
        # sum; for a non-convex one the point matters (parity vs MuJoCo unpinned: its source is absent)
        a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
        area = 0.5 * np.linalg.norm(np.cross(b - a, c - a), axis=1)
        ref = (area[:, None] * (a + b + c) / 3.0).sum(0) / area.sum()
    else:
        ref = np.zeros(3)
    a, b, c = v[f[:, 0]] - ref, v[f[:, 1]] - ref, v[f[:, 2]] - ref
    vol, cen, cov = _tet_props(a, b, c)
    if mode == "legacy":
        sg = np.sign(vol)
        vol, cov = vol * sg, cov * sg[:, None, None]
    elif mode != "exact":
        raise ValueError(f"unknown mesh inertia mode {mode!r}")
    V = vol.sum()
    if not V > 0:
        raise ValueError("mesh volume is not positive (open or inverted mesh?)")
    com_r = (vol[:, None] * cen).sum(0) / V
    C = cov.sum(0) - V * np.outer(com_r, com_r)   # covariance about the com
    return V, com_r + ref, np.trace(C) * np.eye(3) - C


def principal_frame(I):
    """(diagonal inertia [3], rotation matrix whose columns are the principal axes, det +1)"""
    w, R = np.linalg.eigh(0.5 * (I + I.T))
    if np.linalg.det(R) < 0:
        R[:, 2] = -R[:, 2]
    return w, R
