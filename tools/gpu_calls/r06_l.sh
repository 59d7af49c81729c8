#!/bin/bash
# round-6 GPU call: the per-step RCCL gather (self-gather at one rank) with the env steps on a high-priority
# stream (the product default beside the gather) against a normal-priority one, and no gather, alternated
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
B="python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra --gather-self"
for i in 1 2 3; do
  for v in nogather high normal; do
    X=""; [ $v = nogather ] && X="--no-gather"; [ $v = normal ] && X="--env-priority normal"
    timeout -k 10 300 $B $X > $D/$v$i.json 2> $D/$v$i.err || { echo "$v failed"; tail -5 $D/$v$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$v$i.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,4), round(d['ms_per_step'],4), d['config']['parallelism'], d['config'].get('env_stream_priority'), (d.get('gather') or {}).get('rank0_slot_check'))"
  done
done
