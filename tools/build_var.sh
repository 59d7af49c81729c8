#!/bin/bash
# build the working tree's sources into ur3e_amd/_lib/libur3e_amd_var.so (for tools/ab.sh), leaving the
# product library alone.  usage: tools/build_var.sh [-DNAME ...]
set -e
cd "$(dirname "$0")/.."
# ur3e_mjcf.cpp includes the generated (git-ignored) gen_pyconfig.h and the kernels gen_main_tree.h:
# write them first, so a clean checkout or worktree builds
python3 -c 'from ur3e_amd import _build; _build.gen_pyconfig(); _build.gen_main_tree()'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -disable-machine-licm \
  -Wno-unused-result "$@" -o ur3e_amd/_lib/libur3e_amd_${VAR:-var}.so ur3e_amd/csrc/ur3e_batch.hip ur3e_amd/csrc/ur3e_vecnorm.hip ur3e_amd/csrc/ur3e_mjcf.cpp ur3e_amd/csrc/ur3e_gather.cpp -ldl
