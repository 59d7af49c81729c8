"""The C-ABI library builds for gfx950, loads, and exports every entry point
include/*.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    import glob
    names = set()
    for h in sorted(glob.glob(os.path.join(REPO, "include", "*.h"))):
        src = open(h).read()
        names |= set(re.findall(r"^\s*(?:int|const char\*)\s+(ur3e_\w+)\(", src, re.M))
    return sorted(names)


def test_library_exports_header_symbols():
    from ur3e_amd import _build
    lib = _build.build()
    assert os.path.exists(lib)
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ur3e_\w+)", out))
    decl = _declared()
    assert len(decl) >= 15 and "ur3e_vecnorm_step" in decl
    missing = [s for s in decl if s not in exported]
    assert not missing, missing
    L = ctypes.CDLL(lib)
    assert L.ur3e_abi_version() == 9
    for s in decl:
        getattr(L, s)


def test_code_object_is_gfx950():
    from ur3e_amd import _build
    lib = _build.build()
    data = open(lib, "rb").read()
    assert b"gfx950" in data


def test_model_struct_layout_matches_header():
    """ctypes mirror == C struct: the oracle (plain C) reports its sizeof view through a probe."""
    from ur3e_amd.model.compiler import UR3eModelC
    from ur3e_amd.runtime import ConfigC
    from oracle.pyoracle import OracleConfig
    src = (
        '#include <stdio.h>\n#include <stddef.h>\n#include "include/ur3e_batch.h"\n'
        'int main(){printf("%zu %zu %zu\\n", sizeof(ur3e_model_t), sizeof(ur3e_config_t), '
        'offsetof(ur3e_config_t, rot_joint_gains));return 0;}\n')
    exe = os.path.join(REPO, "oracle", "_build", "sizeof_probe")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    cfile = exe + ".c"
    open(cfile, "w").write(src)
    subprocess.run(["gcc", "-I", REPO, "-o", exe, cfile], check=True)
    n, nc, off = map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split())
    assert n == ctypes.sizeof(UR3eModelC)
    assert nc == ctypes.sizeof(ConfigC) == ctypes.sizeof(OracleConfig)
    assert off == ConfigC.rot_joint_gains.offset
