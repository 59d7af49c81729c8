"""Per-kernel resources read from a built library's gfx950 code object (no GPU needed): VGPRs, AGPRs,
SGPRs, scratch (private segment) bytes per lane, static LDS and the compiler's spill counts, from the
AMDGPU metadata note.  `Batch.kernel_info` joins them to the kernel the handle launches by its symbol;
`tools/kinfo.py` prints them for every kernel."""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
_cache: dict = {}


def kernels(lib: str) -> list:
    """[{name, vgpr, agpr, sgpr, scratch, lds, vgpr_spill, sgpr_spill, args}, ...] of every kernel in `lib`
    (args: the kernarg layout, [{offset, size, value_kind}, ...] in parameter order, hidden arguments last)"""
    key = (os.path.abspath(lib), os.path.getmtime(lib))
    if key in _cache:
        return _cache[key]
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True,
                       capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True,
                       capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                               check=True).stdout
    out, cur, args_ind = [], None, None
    for line in notes.splitlines():
        t = line.strip()
        ind = len(line) - len(line.lstrip())
        m = re.match(r"^- \.agpr_count:\s*(\d+)", t)
        if m:
            cur = {"agpr": int(m.group(1)), "args": []}
            out.append(cur)
            args_ind = None
            continue
        if cur is None:
            continue
        if t == ".args:":
            args_ind = ind
            continue
        if args_ind is not None:
            if ind > args_ind:  # inside the argument list: one "- ." line opens each argument
                if t.startswith("- "):
                    cur["args"].append({})
                    t = t[2:]
                k, _, v = t.partition(":")
                if cur["args"] and k in (".offset", ".size", ".value_kind"):
                    v = v.strip()
                    cur["args"][-1][k[1:]] = int(v) if v.isdigit() else v
                continue
            args_ind = None
        for k, name in ((".name:", "name"), (".vgpr_count:", "vgpr"), (".sgpr_count:", "sgpr"),
                        (".private_segment_fixed_size:", "scratch"), (".group_segment_fixed_size:", "lds"),
                        (".vgpr_spill_count:", "vgpr_spill"), (".sgpr_spill_count:", "sgpr_spill")):
            if t.startswith(k):
                v = t[len(k):].strip()
                cur[name] = int(v) if v.isdigit() else v
    _cache[key] = out
    return out


def resources(lib: str, symbol: str) -> dict | None:
    """the code-object entry of kernel `symbol` (its mangled name, or the .kd descriptor's) in `lib`"""
    if not symbol:
        return None
    sym = symbol[:-3] if symbol.endswith(".kd") else symbol
    for k in kernels(lib):
        if k.get("name") == sym:
            return {x: k[x] for x in ("vgpr", "agpr", "sgpr", "scratch", "vgpr_spill", "sgpr_spill") if x in k}
    return None
