#!/bin/bash
# round-5 GPU call: run-ahead marker every 8 steps (product) against every step (libur3e_amd_var.so,
# -DW_AHEAD_EVERY=1): parity subset on the product, then gap probe and bench alternating -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_record.py tests/test_gpu_queue.py -x -q --timeout 300 --timeout-method thread > $D/parity.txt 2>&1 || { tail -30 $D/parity.txt; exit 1; }
tail -1 $D/parity.txt
for i in 1 2 3; do
  for v in base var; do
    if [ $v = base ]; then unset UR3E_LIB; else export UR3E_LIB=$R/ur3e_amd/_lib/libur3e_amd_var.so; fi
    timeout -k 10 200 python3 tools/gap_probe.py 4096 200 > $D/gap_$v$i.json 2>/dev/null || { echo "gap $v failed"; exit 1; }
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra > $D/bench_$v$i.json 2> $D/bench_$v$i.err || { echo "bench $v failed"; tail -3 $D/bench_$v$i.err; exit 1; }
    python3 -c "import json;g=json.load(open('$D/gap_$v$i.json'));d=json.loads(open('$D/bench_$v$i.json').read().strip().splitlines()[-1]);print('$v',{k:round(x['us_per_step'],1) for k,x in g.items()},'bench',round(d['value']/1e6,4),round(d['ms_per_step']*1e3,1),round(d['roofline']['kernel_ms_instrumented']*1e3,1))"
  done
done
