"""Compile the reference MJCF models into committed JSON model images.

Runs in the build container only (it reads /root/reference/assets/*.xml, which
does not exist on the GPU box).  Output: ur3e_amd/assets/<name>.model.json.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ur3e_amd.model.compiler import compile_mjcf, save_json  # noqa: E402

REF = os.environ.get("UR3E_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(__file__), "..", "ur3e_amd", "assets")

for name in ("main", "ur3e_2f85", "ur3e_raw"):
    m = compile_mjcf(os.path.join(REF, "assets", f"{name}.xml"))
    save_json(m, os.path.join(OUT, f"{name}.model.json"))
    print(name, "nq", m["nq"], "nv", m["nv"], "nu", m["nu"], "nbody", m["nbody"], "ngeom", m["ngeom"],
          "ncpair", m["ncpair"], "neq", m["neq"], "meaninertia", m["meaninertia"])
