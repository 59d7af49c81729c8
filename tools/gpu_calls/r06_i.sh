#!/bin/bash
# round-6 GPU call: same-box A/B of the per-env-step kernels' kernarg view (kstep0 reverts it) and of two
# backend options (early if-conversion; the AMDGPU register-pressure trackers in the scheduler), with the
# other configs
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
AB_EXTRA=1 timeout -k 10 1000 bash tools/ab_multi.sh ${ROUNDS:-2} kstep0 ifcvt trackers 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
