#!/bin/bash
# round-4 GPU call: the GPU suite, then a same-box A/B of the pre-narrowphase cull (plane-mesh clause
# added) with the other configs, into gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?; tail -3 $D/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
AB_EXTRA=1 bash tools/ab_multi.sh 2 cull0 > $D/ab.txt 2>&1; rc=$?; tail -6 $D/ab.txt; [ $rc -eq 0 ] || exit $rc
