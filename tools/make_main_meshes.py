"""Synthetic stand-ins for the mesh files assets/main.xml names (the reference git-ignores them, so its
own model can only run on the box surrogate), so that the real-mesh path (compile_mjcf(meshes="mesh"),
GJK/EPA in ur3e_amd/csrc/convex.h) runs on the reference's full model.

Every mesh becomes a convex "rounded box" hull: points of a Fibonacci sphere pushed onto the surface
{x : sum_k ((x_k - c_k) / h_k)^4 = 1} (convex), where h and c are the mesh's box-surrogate half sizes
and centre (ur3e_amd/model/surrogate.py), written in the mesh's own units (the MJCF scale divided out).
The 2F-85 linkage parts the surrogate makes visual-only (their box stand-ins would collide inside the
linkage; the real parts are shaped not to) are shrunk about their centre until the rest pose of main.xml
shows the surrogate model's contact set (tools/make_main_meshes.py checks that with the oracle).
The hull vertex budget of the model image is UR3E_MAXMESHVERT = 1024 over UR3E_MAXMESH = 16 meshes.

usage: python tools/make_main_meshes.py [OUTDIR]   (writes the meshes under OUTDIR, default
/tmp/ur3e_main_meshes, then ur3e_amd/assets/main_mesh.model.json; needs /root/reference/assets/main.xml)"""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from ur3e_amd.model import mesh as M  # noqa: E402
from ur3e_amd.model.surrogate import MESH_SURROGATE  # noqa: E402

REF = os.environ.get("UR3E_REFERENCE", "/root/reference")
NPTS_COLLIDE = 60
NPTS_VISUAL = 48
SHRINK_NONCOLLIDING = 0.6


def fibonacci(n):
    i = np.arange(n) + 0.5
    phi = np.arccos(1 - 2 * i / n)
    th = np.pi * (1 + 5 ** 0.5) * i
    return np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], axis=1)


def rounded_box(h, c, n):
    d = fibonacci(n)
    p = d / (np.sum(d ** 4, axis=1) ** 0.25)[:, None]
    return np.asarray(c) + p * np.asarray(h)


def write_binary_stl(path, V, F):
    with open(path, "wb") as f:
        f.write(b"ur3e synthetic stand-in mesh".ljust(80, b"\0"))
        f.write(struct.pack("<I", len(F)))
        for t in F:
            p0, p1, p2 = V[t[0]], V[t[1]], V[t[2]]
            n = np.cross(p1 - p0, p2 - p0)
            n = n / (np.linalg.norm(n) or 1.0)
            f.write(struct.pack("<12fH", *n, *p0, *p1, *p2, 0))


def write_meshes(out_dir, main_xml):
    import xml.etree.ElementTree as ET
    from ur3e_amd.model.compiler import _Defaults, _mesh_assets
    root = ET.parse(main_xml).getroot()
    assets = _mesh_assets(root, _Defaults(root), main_xml, out_dir)
    written = {}
    for name, a in assets.items():
        h, c, collide = MESH_SURROGATE[name]
        h = np.asarray(h, float) * (1.0 if collide else SHRINK_NONCOLLIDING)
        V = rounded_box(h, c, NPTS_COLLIDE if collide else NPTS_VISUAL) / np.asarray(a["scale"])
        V = V.astype(np.float32).astype(np.float64)  # what the STL stores
        _, F = M.convex_hull(V)
        os.makedirs(os.path.dirname(a["file"]), exist_ok=True)
        if a["file"].endswith(".obj"):
            M.write_obj(a["file"], V, F)
        else:
            write_binary_stl(a["file"], V, F)
        written[name] = len(V)
    return written


def main(out_dir="/tmp/ur3e_main_meshes"):
    from ur3e_amd.model.compiler import compile_mjcf, save_json
    main_xml = os.path.join(REF, "assets", "main.xml")
    w = write_meshes(out_dir, main_xml)
    md = compile_mjcf(main_xml, meshes="mesh", meshdir=out_dir)
    out = os.path.join(REPO, "ur3e_amd", "assets", "main_mesh.model.json")
    save_json(md, out)
    print(f"{len(w)} meshes, {sum(w.values())} points -> {md['nmeshvert']} hull vertices; "
          f"ngeom {md['ngeom']}, ncpair {md['ncpair']}, mesh geoms {int(np.sum(np.asarray(md['geom_type']) == 7))}")
    return md


if __name__ == "__main__":
    main(*sys.argv[1:2])
