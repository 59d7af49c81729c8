#!/bin/bash
# round-4 GPU call: same-box A/B of the lane-parallel gym controller/epilogue (epi0 = lane 0 only) and
# the cone-term skip (cone0 = always computed) against the product library, then the GPU suite, smoke and
# the round profile (bench line with CPU baseline and other configs, kernel trace, PMC) into gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
bash tools/ab_multi.sh 2 epi0 cone0 > $D/ab.txt 2>&1; rc=$?; tail -8 $D/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?; tail -3 $D/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit $?
bash tools/profile_round.sh $1
