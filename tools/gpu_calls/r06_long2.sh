#!/bin/bash
# round-6 GPU call (after A/B 9, the Newton Hessian's equality-row prefix): the long GPU-vs-oracle rollouts at the head for both compiles (gym 4,096 x 3,000 every
# step; the C3 scripted pick 1,024 x 4,200 rows through grasp, lift and carry, which takes the mid tier) -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
for M in main_mesh main; do
  timeout -k 10 500 python3 -u tools/long_parity.py 4096 3000 $M > $D/gym_${M}_4096x3000.json 2> $D/gym_$M.err || { tail -5 $D/gym_$M.err; exit 1; }
  tail -c 600 $D/gym_${M}_4096x3000.json; echo
  timeout -k 10 500 python3 -u tools/long_parity_c3.py 1024 4200 300 $M > $D/c3_${M}_1024x4200.jsonl 2> $D/c3_$M.err || { tail -5 $D/c3_$M.err; exit 1; }
  tail -2 $D/c3_${M}_1024x4200.jsonl | cut -c1-400
done
