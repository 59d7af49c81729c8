#!/bin/bash
# round-4 GPU call: same-box A/B of the full-capacity tier's launch grid (512 default, 128, 32), gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
bash tools/ab_multi.sh 3 full128 full32 > $D/ab.txt 2>&1; rc=$?; tail -9 $D/ab.txt; [ $rc -eq 0 ] || exit $rc
