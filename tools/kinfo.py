"""Build-side diagnostic (no GPU): per-kernel resources of a built library's gfx950 code object -- VGPRs,
AGPRs, SGPRs, scratch (private segment) bytes per lane, static LDS -- read from the code object's AMDGPU
metadata note.  usage: python tools/kinfo.py [lib.so] [name-regex]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(lib):
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        t = line.strip()
        m = re.match(r"^- \.agpr_count:\s*(\d+)", t)
        if m:
            cur = {"agpr": int(m.group(1))}
            out.append(cur)
            continue
        if cur is None:
            continue
        for key, name in ((".name:", "name"), (".vgpr_count:", "vgpr"), (".sgpr_count:", "sgpr"),
                          (".private_segment_fixed_size:", "scratch"), (".group_segment_fixed_size:", "lds"),
                          (".vgpr_spill_count:", "vgpr_spill"), (".sgpr_spill_count:", "sgpr_spill")):
            if t.startswith(key):
                v = t[len(key):].strip()
                cur[name] = int(v) if v.isdigit() else v
    return out


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
