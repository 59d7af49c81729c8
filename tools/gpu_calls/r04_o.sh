#!/bin/bash
# round-4 GPU call: the head build's queue trace and lane-0 stage timing (diagnostic builds), gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 300 python3 -u tools/queue_trace.py 4096 4 > $D/qtrace.txt 2>&1 || exit $?
tail -1 $D/qtrace.txt
timeout -k 10 300 python3 -u tools/stage_timing.py 4096 0 gym 0 > $D/stage_gym.txt 2>&1 || exit $?
tail -3 $D/stage_gym.txt
