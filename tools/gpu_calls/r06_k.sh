#!/bin/bash
# round-6 GPU call: the per-step RCCL gather with the env step writing into the payload (no packing kernels,
# event-precise double buffering) against no gather, at one rank (self-gather), alternated twice; plus the
# step-into-buffers test -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step_out.py tests/test_gpu_gather_rccl.py -x -q --timeout 200 --timeout-method thread > $D/tests.txt 2>&1 || { tail -30 $D/tests.txt; exit 1; }
tail -1 $D/tests.txt
B="python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra --gather-self"
for i in 1 2; do
  for v in nogather gather; do
    X=""; [ $v = nogather ] && X="--no-gather"
    timeout -k 10 300 $B $X > $D/$v$i.json 2> $D/$v$i.err || { echo "$v failed"; tail -5 $D/$v$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$v$i.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,4), round(d['ms_per_step'],4), d['config']['parallelism'], d.get('gather'))"
  done
done
