#!/bin/bash
# round-5 GPU call: the mesh model at HEAD -- gym bench line, kernel trace, C3 windows on both compiles
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 python3 bench.py --model main_mesh --no-cpu-baseline > $D/bench_mesh.json 2> $D/bench_mesh.err || exit $?
tail -1 $D/bench_mesh.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --model main_mesh --steps 50 --warmup 5 --no-cpu-baseline > $D/trace.log 2>&1 || exit $?
head -5 $D/trace/run_kernel_stats.csv | cut -c1-300
timeout -k 10 400 python3 -u tools/mesh_c3.py 4096 > $D/mesh_c3.txt 2>&1 || exit $?
cat $D/mesh_c3.txt | cut -c1-300
