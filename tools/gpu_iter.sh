#!/bin/bash
# one GPU iteration: parity (fast set), throughput, per-stage cycles.  Usage: tools/gpu_iter.sh OUTDIR
set -o pipefail
D=gpurun_out/$1
mkdir -p $D
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "not 1000" > $D/parity.log 2>&1
rc=$?
tail -3 $D/parity.log
[ $rc -ne 0 ] && { tail -40 $D/parity.log; exit $rc; }
timeout -k 10 200 python tools/epb_sweep.py 4096 ${EPB:-0} > $D/epb.log 2>&1 || exit $?
cat $D/epb.log | tail -1
if [ -f ur3e_amd/_lib/libur3e_amd_timing.so ]; then
  timeout -k 10 200 python tools/stage_timing.py 4096 0 > $D/stages.log 2>&1 || exit $?
  cat $D/stages.log
fi
