#!/bin/bash
# round-4 GPU call: same-box A/B of the pre-narrowphase cull (cull0 = off) against the product library,
# the GPU suite, smoke and the round profile into gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1
rc=$?; tail -3 $D/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
AB_EXTRA=1 bash tools/ab_multi.sh 2 cull0 > $D/ab.txt 2>&1; rc=$?; tail -6 $D/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit $?
bash tools/profile_round.sh $1
