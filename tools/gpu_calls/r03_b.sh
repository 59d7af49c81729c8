set -o pipefail
D=gpurun_out/r03_b; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_c3_record.py tests/test_gpu_c5_policy.py tests/test_gpu_config.py tests/test_gpu_queue.py -x -v -s --timeout 200 --timeout-method thread > $D/new_tests.txt 2>&1 || { tail -40 $D/new_tests.txt; exit 1; }
grep -E "PASS|FAIL|grasp flag" $D/new_tests.txt | tail -10
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
bash tools/r03_analysis.sh
