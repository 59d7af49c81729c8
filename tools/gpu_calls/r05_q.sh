#!/bin/bash
# round-5 GPU call: parity of the passive, actuator and connect plan rows (product library), then same-box A/B against the
# the previous commit (libur3e_amd_var.so built from HEAD) on both models
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mesh_main.py tests/test_gpu_mesh_c3.py tests/test_gpu_c3_record.py tests/test_gpu_touch.py -x -q --timeout 300 --timeout-method thread > $D/parity.txt 2>&1 || { tail -40 $D/parity.txt; exit 1; }
tail -1 $D/parity.txt
AB_TAG=_main bash tools/ab.sh 3 || exit $?
AB_TAG=_mesh AB_ARGS="--model main_mesh" bash tools/ab.sh 3 || exit $?
