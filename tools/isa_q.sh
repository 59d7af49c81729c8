#!/bin/bash
# Device ISA of the working tree's compact-tier queue kernel (gym model, production template) for
# static instruction comparisons: tools/isa_q.sh NAME [-DFLAG ...] -> /tmp/isa/NAME.s, /tmp/isa/NAME_q.s
set -e
cd "$(dirname "$0")/.."
N=$1; shift
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm \
  --cuda-device-only -S -Iinclude "$@" -o /tmp/isa/$N.s ur3e_amd/csrc/ur3e_batch.hip
python3 - /tmp/isa/$N.s /tmp/isa/${N}_q.s <<'PY'
import sys, re
src = open(sys.argv[1]).read().split('\n')
out, on = [], False
for l in src:
    if re.match(r'^_Z12w_env_step_qILi64E3KSXILi10ELi44ELi20ELi1ELb1EELin1EE[^:]*:', l): on = True
    if on:
        out.append(l)
        if l.startswith('.Lfunc_end'): break
open(sys.argv[2], 'w').write('\n'.join(out))
n = sum(1 for l in out if l.strip().startswith('v_'))
print(sys.argv[2], 'lines', len(out), 'VALU', n)
PY
