#!/bin/bash
# round-4 GPU call: the long GPU-vs-oracle rollouts at the head build (gym 4,096 x 3,000 every step;
# the C3 scripted pick 1,024 x 3,000 rows through grasp and lift), then a same-box A/B of the full-capacity
# tier launch grid (512, 128, 32), into gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 900 python3 -u tools/long_parity.py 4096 3000 > $D/gym_4096x3000.json 2> $D/gym.err || exit $?
cat $D/gym_4096x3000.json
timeout -k 10 900 python3 -u tools/long_parity_c3.py 1024 3000 > $D/c3_move_l_mug_1024x3000.jsonl 2> $D/c3.err || exit $?
tail -2 $D/c3_move_l_mug_1024x3000.jsonl
bash tools/ab_multi.sh 3 full128 full32 > $D/ab_fullgrid.txt 2>&1; rc=$?; tail -9 $D/ab_fullgrid.txt; [ $rc -eq 0 ] || exit $rc
