#!/bin/bash
# round-6 GPU call: the GPU suite with the mid tier (16 contacts / 64 rows between the compact and the grasp
# tier), the C3 mesh pick window by window, then same-box A/B against the three-tier chain (mid0) with the
# other configs (C3 on both compiles)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -1 $D/gpu_tests.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mesh_c3.py -q -s --timeout 300 --timeout-method thread > $D/mesh_c3_test.txt 2>&1 || { tail -20 $D/mesh_c3_test.txt; exit 1; }
grep "tier counts" $D/mesh_c3_test.txt
timeout -k 10 300 python3 tools/mesh_c3.py 4096 main_mesh,main > $D/c3_windows.jsonl 2> $D/c3_windows.err || { tail -5 $D/c3_windows.err; exit 1; }
cut -c1-260 $D/c3_windows.jsonl
AB_EXTRA=1 timeout -k 10 700 bash tools/ab_multi.sh ${ROUNDS:-2} mid0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
