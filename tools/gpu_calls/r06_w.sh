#!/bin/bash
# round-6 GPU call: a second Newton-Hessian prefix over every non-contact row, reused while their quadratic set is
# unchanged (W_HB_NC_PRE): the C3 diagnostic per layout, the GPU suite, then the same-box A/B against ncpre0
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 python3 -u tools/dbg_c3_tiers.py default full128 cap3 > $D/c3_layouts.txt 2>&1 || { tail -20 $D/c3_layouts.txt; exit 1; }
grep mismatch $D/c3_layouts.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
AB_EXTRA=1 timeout -k 10 800 bash tools/ab_multi.sh ${ROUNDS:-2} ncpre0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
