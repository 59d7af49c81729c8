#!/bin/bash
# round-6 GPU call: raw unit timeline of the mesh headline's queue kernel (trace build, env-steps 500-507) for
# the offline model of unit orders (tools/lpt_sim.py)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
UR3E_TRACE_MODEL=main_mesh UR3E_TRACE_PRE=500 UR3E_TRACE_OUT=$D/trace.npz timeout -k 10 300 python3 -u tools/queue_trace.py 4096 8 > $D/trace.txt 2>&1 || { tail -20 $D/trace.txt; exit 1; }
grep -v warm-up $D/trace.txt
python3 tools/lpt_sim.py $D/trace.npz | tee $D/lpt_sim.txt
