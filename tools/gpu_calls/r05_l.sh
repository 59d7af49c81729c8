#!/bin/bash
# round-5 GPU call: the host/launch share of the gym env-step (tools/gap_probe.py), then a kernel trace
# of the probe to read the gaps between launches -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 200 python3 -u tools/gap_probe.py 4096 200 > $D/gap_probe.json 2> $D/gap_probe.err || { tail -20 $D/gap_probe.err; exit 1; }
cat $D/gap_probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/trace -o run -- python3 tools/gap_probe.py 4096 200 > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
ls $D/trace
