"""The mesh variant of the reference's model (ur3e_amd/assets/main_mesh.model.json): assets/main.xml compiled
with real convex mesh geoms from synthetic stand-in hulls (tools/make_main_meshes.py; the reference ships
no mesh files).  CPU checks: the committed image is what the generator produces from the reference's
main.xml (when the checkout is present), it stays within the image capacities, and on the oracle it rests
with the surrogate model's contact set and has the same kind of constraint rows under random gym actions."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_MAIN = "/root/reference/assets/main.xml"


def test_image_capacities():
    from ur3e_amd import runtime as rt
    md, _ = rt.load_model("main_mesh")
    gt = np.asarray(md["geom_type"][:md["ngeom"]])
    assert md["ngeom"] == 24 and int((gt == 7).sum()) == 17
    assert md["nmesh"] <= 16 and md["nmeshvert"] <= 1024
    assert md["ncpair"] <= 240  # W_MAXCAND_MESH (ur3e_amd/csrc/ur3e_wave.h)
    ms, _ = rt.load_model("main")
    for k in ("nq", "nv", "nu", "nbody", "njnt", "nsite"):
        assert md[k] == ms[k], k


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="reference checkout absent (GPU box)")
def test_committed_image_regenerates(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_main_meshes as mm
    from ur3e_amd.model.compiler import compile_mjcf, load_json, to_ctypes
    mm.write_meshes(str(tmp_path), REF_MAIN)
    md = compile_mjcf(REF_MAIN, meshes="mesh", meshdir=str(tmp_path))
    committed = load_json(os.path.join(ROOT, "ur3e_amd", "assets", "main_mesh.model.json"))
    assert bytes(to_ctypes(md)) == bytes(to_ctypes(committed))


def test_rest_contacts_and_rows_match_the_surrogate():
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    out = {}
    for name in ("main", "main_mesh"):
        md, mc = rt.load_model(name)
        d = po.OracleData(mc)
        d.set(qpos=np.array(md["key_qpos"][md["id_key_down"]]), qvel=np.zeros(md["nv"]))
        d.forward()
        c = d.contacts()
        gn = md["geom_names"]
        rest = sorted((gn[a], gn[b]) for a, b in c["geoms"])
        cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=5)
        ob = po.OracleBatch(mc, po.config_from(cfg), 32)
        rng = np.random.default_rng(0)
        lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
        hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
        rows = []
        for t in range(60):
            ob.step(rng.uniform(lo, hi, size=(32, 4)))
            if t % 10 == 9:
                rows += [ob.diag(i)["nefc"] for i in range(32)]
        out[name] = (rest, np.bincount(rows, minlength=64))
    assert out["main"][0] == out["main_mesh"][0] == [("table", "fish")] * 4
    # the mesh inertias change the motion, not the kind of contact: 4 mug-table contacts (13 + 12 rows)
    # plus the odd joint-limit row in both
    for name in ("main", "main_mesh"):
        h = out[name][1]
        assert h[:25].sum() == 0 and h[28:].sum() == 0 and h[25] > h[26:28].sum(), (name, np.nonzero(h))
