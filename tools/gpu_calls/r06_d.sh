#!/bin/bash
# round-6 GPU call: same-box A/B of the mesh broadphase's pair constants loaded ahead (product) against per
# pass (tools/var/broad0.flags), then the queue trace of the mesh headline mid-episode (span vs ideal)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 900 bash tools/ab_multi.sh ${ROUNDS:-4} broad0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
UR3E_TRACE_MODEL=main_mesh UR3E_TRACE_PRE=500 timeout -k 10 300 python3 tools/queue_trace.py 4096 4 > $D/queue_trace.jsonl 2> $D/queue_trace.err || { tail -5 $D/queue_trace.err; exit 1; }
tail -4 $D/queue_trace.jsonl
