#!/bin/bash
# round-6 final GPU call: the GPU suite, smoke, and the profiles of the head for both compiles of main.xml
# (bench line, kernel trace, HBM and SQ counters) -> gpurun_out/$1/{mesh,main}
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { cat $D/smoke.txt; exit 1; }
tail -1 $D/smoke.txt
bash tools/profile_round.sh $1/mesh || exit $?
bash tools/profile_round.sh $1/main --model main --no-extra || exit $?
