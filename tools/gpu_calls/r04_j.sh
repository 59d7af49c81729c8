#!/bin/bash
# round-4 GPU call: the GPU suite, then a same-box A/B of pulling the next queue unit ahead (ahead0 = off)
# and the queue trace of the build, into gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?; tail -3 $D/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_multi.sh 3 ahead0 mid0 > $D/ab.txt 2>&1; rc=$?; tail -7 $D/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/queue_trace.py 4096 4 > $D/qtrace.txt 2>&1 || exit $?
tail -2 $D/qtrace.txt
