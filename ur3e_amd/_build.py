"""Build the MI355X HIP library in-tree: ur3e_amd/_lib/libur3e_amd.so (gfx950)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "ur3e_batch.hip")
DEPS = [SRC, os.path.join(HERE, "csrc", "ur3e_engine.h"), os.path.join(HERE, "csrc", "ur3e_wave.h"), os.path.join(HERE, "csrc", "ur3e_wave_r.h"),
        os.path.join(HERE, "csrc", "detmath.h"),
        os.path.join(HERE, "..", "include", "ur3e_model.h"), os.path.join(HERE, "..", "include", "ur3e_batch.h")]
LIB = os.path.join(HERE, "_lib", "libur3e_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wno-unused-result"]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not force and os.path.exists(LIB):
        t = os.path.getmtime(LIB)
        if all(os.path.getmtime(d) <= t for d in DEPS):
            return LIB
    cmd = [HIPCC] + FLAGS + ["-o", LIB, SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    build(force=True, verbose=True)
