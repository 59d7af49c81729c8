set -o pipefail
D=gpurun_out/r03_an; mkdir -p $D
UR3E_TRACE_OUT=$D/q4096.npz timeout -k 10 200 python3 tools/queue_trace.py 4096 4 > $D/qtrace.log 2>&1 || { tail -20 $D/qtrace.log; exit 1; }
tail -2 $D/qtrace.log
python3 tools/pair_divergence.py $D/q4096.npz > $D/pair_divergence.json && cat $D/pair_divergence.json | tail -3
timeout -k 10 60 rocprofv3 --list-avail > $D/avail.txt 2>&1 || true
bash tools/stage_classes.sh r03_stage
