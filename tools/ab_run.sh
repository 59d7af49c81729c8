#!/bin/bash
# GPU: parity of the variant library (GPU tests on it), then same-box A/B against the product library
set -o pipefail
D=gpurun_out/ab; mkdir -p $D
UR3E_LIB=$PWD/ur3e_amd/_lib/libur3e_amd_var.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py -x -q --timeout 200 --timeout-method thread -k "not 1000 and not trace" > $D/var_parity.txt 2>&1 || { tail -30 $D/var_parity.txt; exit 1; }
tail -1 $D/var_parity.txt
bash tools/ab.sh ${1:-3}
