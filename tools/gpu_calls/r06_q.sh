#!/bin/bash
# round-6 GPU call: same-box A/B of the full-capacity tier's grid (512 workgroups of 80 KB LDS dispatched every
# step for the route snapshot and a nearly always empty list) at 64 and 128
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
AB_EXTRA=1 timeout -k 10 1000 bash tools/ab_multi.sh ${ROUNDS:-2} fg64 fg128 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
