#!/bin/bash
# round-5 GPU call: lane-0 stage timing mid-episode (500 env-steps from reset) on both compiles of main.xml;
# the two-envs-per-wave microbenchmark (tools/ubench_halfwave.hip)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 120 ./tools/ubench_halfwave 4096 16 > $D/halfwave_4096.txt 2>&1 || { cat $D/halfwave_4096.txt; exit 1; }
cat $D/halfwave_4096.txt
timeout -k 10 120 ./tools/ubench_halfwave 16384 16 > $D/halfwave_16384.txt 2>&1 || { cat $D/halfwave_16384.txt; exit 1; }
cat $D/halfwave_16384.txt
for m in main_mesh main; do
  for pre in 3 500; do
    UR3E_STAGE_MODEL=$m UR3E_STAGE_PRE=$pre timeout -k 10 300 python3 -u tools/stage_timing.py 4096 0 gym 0 > $D/stage_${m}_pre$pre.txt 2>&1 || exit $?
  done
done
for f in $D/stage_*.txt; do echo $f; grep -E "^(39|48|49| 4| 5|10|20|total)" $f; done
