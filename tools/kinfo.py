"""Build-side diagnostic (no GPU): per-kernel resources of a built library's gfx950 code object -- VGPRs,
AGPRs, SGPRs, scratch (private segment) bytes per lane, static LDS -- read from the code object's AMDGPU
metadata note.  usage: python tools/kinfo.py [lib.so] [name-regex]"""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ur3e_amd.codeobj import kernels  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "ur3e_amd", "_lib",
                                                              "libur3e_amd.so")
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    for k in kernels(lib):
        name = k.get("name", "?")
        if pat and not pat.search(name):
            continue
        print(f"{k.get('vgpr', '?'):>4} vgpr {k.get('agpr', 0):>3} agpr {k.get('sgpr', '?'):>4} sgpr "
              f"{k.get('scratch', '?'):>6} scratch {k.get('lds', '?'):>6} lds "
              f"spill v{k.get('vgpr_spill', '?')}/s{k.get('sgpr_spill', '?')}  {name}")


if __name__ == "__main__":
    main()
