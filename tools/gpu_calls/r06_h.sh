#!/bin/bash
# round-6 GPU call: per-stage cycles (r06_g), the wait breakdown of the headline kernel (r06_wait) and the long
# GPU-vs-oracle rollouts (r06_long) at the head, one box -> gpurun_out/$1/{stages,wait,long}
set -o pipefail
bash tools/gpu_calls/r06_g.sh $1/stages || exit $?
bash tools/gpu_calls/r06_wait.sh $1/wait || exit $?
bash tools/gpu_calls/r06_long.sh $1/long || exit $?
