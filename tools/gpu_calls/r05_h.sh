#!/bin/bash
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5_policy.py -x -q -k "vecnorm or c5 or policy" --timeout 500 --timeout-method thread > $D/vn_tests.txt 2>&1 || { tail -40 $D/vn_tests.txt; exit 1; }
tail -1 $D/vn_tests.txt
timeout -k 10 120 python3 -u tools/vecnorm_blocks.py 4096 > $D/vn_blocks.txt 2>&1 || exit $?
grep -v amdgpu.ids $D/vn_blocks.txt
timeout -k 10 120 python3 -u tools/vecnorm_trace.py 4096 64 > $D/vecnorm.txt 2>&1 || exit $?
grep -v amdgpu.ids $D/vecnorm.txt
