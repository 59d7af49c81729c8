#!/bin/bash
# round-6 GPU call: GPU suite, smoke, the --gpus 2 refusal on a one-GPU box, and the headline profile
# (main_mesh default: bench line, kernel trace, HBM and SQ counters) -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { cat $D/smoke.txt; exit 1; }
tail -1 $D/smoke.txt
# more ranks than GPUs: must fail before any rank starts (no silent one-rank line)
timeout -k 10 120 python3 bench.py --gpus 2 --steps 2 > $D/gpus2.out 2> $D/gpus2.err; echo "gpus2 rc=$?" | tee $D/gpus2.rc
test ! -s $D/gpus2.out || { echo "gpus2 printed a line"; exit 1; }
bash tools/profile_round.sh $1/mesh || exit $?
