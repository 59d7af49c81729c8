set -o pipefail
mkdir -p gpurun_out/r03_base
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_base/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r03_base/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03_base/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_base/smoke.txt 2>&1 || exit 1
bash tools/profile_round.sh r03_base
