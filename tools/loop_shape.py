"""Build-side check of the substep queue kernel's loop shape (no GPU).

The queue kernel (w_env_step_q) relies on wave-uniform control flow around its lane-0 regions: lane 0
pulls a unit / polls a flag and publishes the result in LDS, and the whole wave reads it back after a
wave barrier.  A round-2 trace build whose stamp stores sat under `if (tid == 0)` inside the queue loop
compiled that loop as a divergent two-level nest (the unit pull in an outer loop, the unit body in an
inner loop whose exits are tracked per lane by exec masks) and faulted or hung on its first launch.
In the nest the flag-poll spin loop sits one level deeper (depth 3 instead of 2).

This compiles ur3e_batch.hip to gfx950 assembly with the product flags plus the given -D flags and
prints, for the gym-specialised queue kernel, the loop depth of the flag-poll loop (the one holding
`s_sleep 2`) and of the queue loop header.  A uniform queue loop has the poll at depth 2.
usage: python tools/loop_shape.py [-DNAME ...] [--src FILE] [--expect-depth 2]"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def queue_kernel_asm(src, defs):
    from ur3e_amd import _build
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        flags = [f for f in _build.FLAGS if f not in ("-fPIC", "-shared")]
        subprocess.run([_build.HIPCC] + flags + ["--cuda-device-only", "-S", "-I", os.path.join(REPO, "include"),
                        "-I", os.path.dirname(src)] + defs + ["-o", out, src], check=True)
        text = open(out).read()
    m = re.search(r"^(_Z12w_env_step_qILi64E3KSX\w*?ELi0EEv\w*):", text, re.M)
    if not m:
        raise SystemExit("gym queue kernel not found")
    body = text[m.start():]
    return m.group(1), body[:body.index(".Lfunc_end")]


def poll_depth(body):
    """Depth of the loop that contains the flag poll's s_sleep 2 (from the block annotations)."""
    depth, out = 0, []
    for line in body.splitlines():
        d = re.search(r"Depth=(\d+)", line)
        if d and (":" in line.split(";")[0] or line.strip().startswith(";")):
            depth = int(d.group(1))
        if re.match(r"\s*s_sleep 2\b", line):
            out.append(depth)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    src = os.path.join(REPO, "ur3e_amd", "csrc", "ur3e_batch.hip")
    expect = None
    defs = []
    i = 0
    while i < len(args):
        if args[i] == "--src":
            src = args[i + 1]; i += 2
        elif args[i] == "--expect-depth":
            expect = int(args[i + 1]); i += 2
        else:
            defs.append(args[i]); i += 1
    name, body = queue_kernel_asm(src, defs)
    depths = poll_depth(body)
    print(f"{os.path.relpath(src, REPO) if src.startswith(REPO) else src} {' '.join(defs) or '(product flags)'}: "
          f"flag-poll loop depth {sorted(set(depths))}, ISA lines {body.count(chr(10))}")
    if expect is not None and set(depths) != {expect}:
        raise SystemExit(f"queue loop is nested: flag-poll depth {sorted(set(depths))} != {expect}")
