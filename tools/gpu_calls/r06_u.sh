#!/bin/bash
# round-6 GPU call: the multi-rank paths at the final head on the one-GPU box -- the RCCL gather through a
# self-gather at one rank (--gather-self) and the launcher with two ranks sharing the GPU over gloo
# (--rehearse-shared-gpu); --gpus 2 without the rehearsal must exit 2 with an empty stdout
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 python3 bench.py --gather-self --no-cpu-baseline --no-extra > $D/gather_self.json 2> $D/gather_self.err || { tail -20 $D/gather_self.err; exit 1; }
tail -1 $D/gather_self.json | cut -c1-400
timeout -k 10 400 python3 bench.py --gpus 2 --rehearse-shared-gpu --no-cpu-baseline --no-extra > $D/rehearse2.json 2> $D/rehearse2.err || { tail -20 $D/rehearse2.err; exit 1; }
tail -1 $D/rehearse2.json | cut -c1-400
rc=0; timeout -k 10 120 python3 bench.py --gpus 2 > $D/gpus2.out 2> $D/gpus2.err || rc=$?
echo "gpus2 exit $rc, stdout bytes $(wc -c < $D/gpus2.out)"
