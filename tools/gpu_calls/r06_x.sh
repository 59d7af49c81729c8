#!/bin/bash
# round-6 GPU call: the GPU suite and smoke on the final library (rebuilt after A/B 11's revert; ISA identical to
# the build profiled in r06_final3)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { cat $D/smoke.txt; exit 1; }
tail -1 $D/smoke.txt
timeout -k 10 400 python3 bench.py --no-extra > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
tail -1 $D/bench.json | cut -c1-200
