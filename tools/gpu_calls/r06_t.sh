#!/bin/bash
# round-6 GPU call: same-box A/B of the product (the Newton Hessian's equality-row prefix, round-6 layout) against
# the round-6 final profile's kernels (r06f: the kernel sources of a81d8bf) and against eqpre0 -- is the 3 % lower
# headline of the last boxes the boxes or the code?
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
AB_EXTRA=1 timeout -k 10 1050 bash tools/ab_multi.sh ${ROUNDS:-2} r06f eqpre0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
