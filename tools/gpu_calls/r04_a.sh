#!/bin/bash
# round-4 GPU call A: the GPU test suite on the working tree's library, then a same-box A/B of the
# pending variants (tools/ab_multi.sh).  usage: tools/r04_a.sh ROUNDS VARIANT...
set -o pipefail
R=$(pwd); D=$R/gpurun_out/r04_a; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?; tail -3 $D/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_multi.sh "$@"
