set -o pipefail
D=gpurun_out/r03_queue; mkdir -p $D
timeout -k 10 240 python -u -m pytest tests/test_gpu_queue.py -x -v -s --timeout 120 --timeout-method thread -k "not trace" > $D/queue.txt 2>&1 || { tail -40 $D/queue.txt; exit 1; }
tail -8 $D/queue.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_queue.py -x -v -s --timeout 120 --timeout-method thread -k "trace" > $D/trace.txt 2>&1 || { tail -40 $D/trace.txt; exit 1; }
tail -4 $D/trace.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -30 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
timeout -k 10 300 python3 bench.py --no-extra > $D/bench.json 2> $D/bench.err || exit 1
python3 -c "import json;d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['parity'])"
