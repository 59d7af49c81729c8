#!/bin/bash
# round-4 GPU call: the GPU test suite, smoke, and the default bench line into gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $D/gpu_tests.txt 2>&1
rc=$?; grep -E "passed|failed|error" $D/gpu_tests.txt | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $D/bench.json 2> $D/bench.err || exit $?
tail -c 600 $D/bench.json
