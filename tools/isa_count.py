"""Static instruction counts of the step kernels (build-side diagnostic, no GPU): compiles
ur3e_batch.hip to gfx950 assembly with the product flags (plus any -D given) and prints, per
kernel, the number of VALU / SALU / LDS / VMEM / branch instructions in its body, and its VGPR,
SGPR and LDS figures. Loops are unrolled in these kernels, so a change that removes instructions
from a stage shows up here before any GPU run.
usage: python tools/isa_count.py [-DNAME[=V] ...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main(defs):
    from ur3e_amd import _build
    flags = [f for f in _build.FLAGS if f not in ("-shared", "-fPIC")]
    src = os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_batch.hip")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run([_build.HIPCC] + flags + defs + ["--cuda-device-only", "-S", "-o", out, src], check=True)
        text = open(out).read()
    kern = None
    counts = collections.defaultdict(collections.Counter)
    meta = {}
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            kern = m.group(1)
            continue
        if kern is None:
            continue
        t = line.strip()
        if t.startswith(".Lfunc_end"):
            kern = None
            continue
        m = re.match(r"^;\s*(NumVgprs|NumSgprs|ScratchSize|Occupancy|NumAgprs):\s*(\d+)", t)
        if m:
            meta.setdefault(kern, {})[m.group(1)] = int(m.group(2))
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        counts[kern][classify(t.split()[0])] += 1
    for k, c in counts.items():
        if "w_env_step" not in k:
            continue
        name = re.sub(r"^_Z\d+", "", k)[:40]
        print(f"{name:40s} valu {c['valu']:6d} salu {c['salu']:5d} lds {c['lds']:5d} vmem {c['vmem']:4d} "
              f"br {c['branch']:5d}  {meta.get(k, {})}")


if __name__ == "__main__":
    main(sys.argv[1:])
