#!/bin/bash
# round-6 GPU call: the GPU suite (with the mid tier's bail chain and step-into-buffers tests), then same-box
# A/B of the compact tier's bails straight to the full-capacity tier while routing is on (direct0 reverts it)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
AB_EXTRA=1 timeout -k 10 800 bash tools/ab_multi.sh ${ROUNDS:-2} direct0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
