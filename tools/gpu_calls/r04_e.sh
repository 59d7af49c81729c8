#!/bin/bash
# round-4 GPU call: split last-substep units -- the queue tests first, then the whole GPU suite, the
# queue trace at 0 / 50 / 100 % split, and a same-box bench A/B of the split percentages (gpurun_out/$1)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 300 --timeout-method thread -s > $D/queue_tests.txt 2>&1
rc=$?; grep -E "passed|failed|error" $D/queue_tests.txt | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $D/gpu_tests.txt 2>&1
rc=$?; grep -E "passed|failed|error" $D/gpu_tests.txt | tail -3; [ $rc -eq 0 ] || exit $rc
for p in 0 50 100; do
  UR3E_SPLIT=$p timeout -k 10 300 python3 -u tools/queue_trace.py 4096 4 > $D/qtrace_$p.txt 2>&1 || exit $?
  echo "split $p: $(tail -1 $D/qtrace_$p.txt)"
done
for i in 1 2; do
  for p in 0 25 50 100; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra --queue-split $p > $D/bench_s${p}_$i.json 2> $D/bench_s${p}_$i.err || exit $?
    python3 -c "import json;d=json.loads(open('$D/bench_s${p}_$i.json').read().strip().splitlines()[-1]);print('split $p', round(d['value']/1e6,4), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
  done
done
timeout -k 10 300 python3 -u tools/stage_timing.py 4096 0 gym 0 > $D/stage_gym.txt 2>&1 || exit $?
tail -40 $D/stage_gym.txt
