#!/bin/bash
# round-6 GPU call: the GPU suite on the working-tree library (queue kernel reading its arguments through
# the kernarg pointer; the mesh grasp tier at 18 contacts / 72 rows, two waves per SIMD; the mesh broadphase's
# pair constants loaded ahead), then same-box A/B against each change reverted (tools/var/karg0.flags,
# grasp24.flags), with the other configs (C3 mesh)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
AB_EXTRA=1 timeout -k 10 900 bash tools/ab_multi.sh ${ROUNDS:-2} karg0 grasp24 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
