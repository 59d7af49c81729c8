#!/bin/bash
# round-6 GPU call: the Newton Hessian build skipping the first-tree element slot for chunks of quadratic
# second-tree rows (W_T2_SKIP) and keeping its equality-row prefix across the directions of a solve (W_HB_EQ_PRE):
# the C3 diagnostic per layout, the GPU suite, then the same-box A/B against each off
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 python3 -u tools/dbg_c3_tiers.py default full128 cap3 > $D/c3_layouts.txt 2>&1 || { tail -20 $D/c3_layouts.txt; exit 1; }
grep mismatch $D/c3_layouts.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
AB_EXTRA=1 timeout -k 10 1000 bash tools/ab_multi.sh ${ROUNDS:-2} t2skip0 eqpre0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
