#!/bin/bash
# round-5 GPU call: wide mesh compact tier for the scripted pick; lane-0 stage timing of the mesh gym step
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mesh_main.py tests/test_gpu_mesh_c3.py -x -v -s --timeout 500 --timeout-method thread > $D/mesh_tests.txt 2>&1 || { tail -40 $D/mesh_tests.txt; exit 1; }
grep -E "passed|failed|tier counts" $D/mesh_tests.txt
timeout -k 10 400 python3 -u tools/mesh_c3.py 4096 main_mesh > $D/mesh_c3.txt 2>&1 || exit $?
cut -c1-250 $D/mesh_c3.txt
UR3E_STAGE_MODEL=main_mesh timeout -k 10 300 python3 -u tools/stage_timing.py 4096 0 gym 0 > $D/stage_mesh_gym.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/stage_timing.py 4096 0 gym 0 > $D/stage_gym.txt 2>&1 || exit $?
paste $D/stage_mesh_gym.txt $D/stage_gym.txt | cut -c1-200
