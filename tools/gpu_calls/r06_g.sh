#!/bin/bash
# round-6 GPU call: per-stage cycles of the mesh headline's compact tier mid-episode (the -DUR3E_STAGE_TIMING
# diagnostic build, libur3e_amd_timing.so built in-tree; read the shares, not the times), both compiles of main.xml
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
UR3E_STAGE_MODEL=main_mesh UR3E_STAGE_PRE=500 timeout -k 10 300 python3 tools/stage_timing.py 4096 0 gym 0 > $D/stage_gym_mesh.txt 2>&1 || { tail -5 $D/stage_gym_mesh.txt; exit 1; }
cat $D/stage_gym_mesh.txt
UR3E_STAGE_MODEL=main UR3E_STAGE_PRE=500 timeout -k 10 300 python3 tools/stage_timing.py 4096 0 gym 0 > $D/stage_gym_main.txt 2>&1 || { tail -5 $D/stage_gym_main.txt; exit 1; }
cat $D/stage_gym_main.txt
