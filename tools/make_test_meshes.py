"""Synthetic mesh assets for the mesh tests (committed under tests/assets/meshes/; test infrastructure):
the main.xml box surrogate of the mug as a triangle mesh (ASCII STL), a unit right tetrahedron (OBJ),
a hexagonal prism (binary STL), and a non-convex L-shaped prism (OBJ, quads) whose MuJoCo 'legacy'
and 'exact' inertia differ.  usage: python tools/make_test_meshes.py"""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from ur3e_amd.model import mesh as M  # noqa: E402

OUT = os.path.join(REPO, "tests", "assets", "meshes")
os.makedirs(OUT, exist_ok=True)

# box with the mug surrogate's half sizes (main.xml:292 geom "fish")
a, b, c = 0.03, 0.02, 0.055111
V = np.array([[sx * a, sy * b, sz * c] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
_, F = M.convex_hull(V)
M.write_stl_ascii(os.path.join(OUT, "box.stl"), V, F)

# unit right tetrahedron, scaled by the MJCF (scale="0.04 0.04 0.04")
T = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1.0]])
_, TF = M.convex_hull(T)
M.write_obj(os.path.join(OUT, "tetra.obj"), T, TF)

# hexagonal prism (radius 0.035, half height 0.04), binary STL
ang = np.arange(6) * np.pi / 3
P = np.array([[0.035 * np.cos(t), 0.035 * np.sin(t), z] for z in (-0.04, 0.04) for t in ang])
_, PF = M.convex_hull(P)
with open(os.path.join(OUT, "prism.stl"), "wb") as f:
    f.write(b"ur3e synthetic hexagonal prism".ljust(80, b"\0"))
    f.write(struct.pack("<I", len(PF)))
    for t in PF:
        p0, p1, p2 = P[t[0]], P[t[1]], P[t[2]]
        n = np.cross(p1 - p0, p2 - p0)
        n = n / np.linalg.norm(n)
        f.write(struct.pack("<12fH", *n, *p0, *p1, *p2, 0))

# L-shaped prism (non-convex): the L in the xy plane extruded along z, quad faces in the OBJ
L2 = np.array([[0, 0], [2, 0], [2, 1], [1, 1], [1, 2], [0, 2]], dtype=float) * 0.01
Lv = np.array([[x, y, z] for z in (0.0, 0.01) for x, y in L2])
faces = []
# bottom (z = 0, outward -z: clockwise seen from above) and top, fanned from vertex 0 of each cap
faces.append("f " + " ".join(str(i + 1) for i in [0, 5, 4, 3, 2, 1]))
faces.append("f " + " ".join(str(i + 7) for i in range(6)))
for i in range(6):
    j = (i + 1) % 6
    faces.append(f"f {i + 1} {j + 1} {j + 7} {i + 7}")
with open(os.path.join(OUT, "lshape.obj"), "w") as f:
    for p in Lv:
        f.write(f"v {p[0]:.17g} {p[1]:.17g} {p[2]:.17g}\n")
    f.write("\n".join(faces) + "\n")
print("wrote", sorted(os.listdir(OUT)))
