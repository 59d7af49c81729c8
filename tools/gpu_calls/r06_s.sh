#!/bin/bash
# round-6 GPU call: same-box A/B of the product (the Newton Hessian's equality-row prefix) against eqpre0, three
# rounds (the final profile's box ran the headline 3 % below round 6's earlier boxes with its wave cycles up 3 %)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
AB_EXTRA=1 timeout -k 10 1000 bash tools/ab_multi.sh ${ROUNDS:-3} eqpre0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
