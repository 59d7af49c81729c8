#!/bin/bash
# round-6 GPU call: the cost of the per-step RCCL gather (obs, reward, done) at one rank (self-gather), against
# no gather, with RCCL's default channel count and with it capped (fewer RCCL workgroups beside the env
# kernel); alternated twice on one box -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
B="python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra --gather-self"
for i in 1 2; do
  for v in nogather default ch1 ch2 ch4; do
    case $v in
      nogather) E=""; X="--no-gather" ;;
      default) E=""; X="" ;;
      ch1) E="NCCL_MAX_NCHANNELS=1"; X="" ;;
      ch2) E="NCCL_MAX_NCHANNELS=2"; X="" ;;
      ch4) E="NCCL_MAX_NCHANNELS=4"; X="" ;;
    esac
    env $E timeout -k 10 300 $B $X > $D/$v$i.json 2> $D/$v$i.err || { echo "$v failed"; tail -5 $D/$v$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$v$i.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,4), round(d['ms_per_step'],4), d['config']['parallelism'])"
  done
done
