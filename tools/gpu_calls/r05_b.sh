#!/bin/bash
# round-5 GPU call: the wavefront convex narrowphase -- mesh parity tests, mesh bench, C3 windows
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mesh_main.py tests/test_gpu_mesh_c3.py tests/test_gpu_mesh.py -x -v -s --timeout 500 --timeout-method thread > $D/mesh_tests.txt 2>&1 || { tail -40 $D/mesh_tests.txt; exit 1; }
grep -E "passed|failed|tier counts" $D/mesh_tests.txt
timeout -k 10 300 python3 bench.py --model main_mesh --no-cpu-baseline > $D/bench_mesh.json 2> $D/bench_mesh.err || exit $?
python3 -c "import json;d=json.loads(open('$D/bench_mesh.json').read().strip().splitlines()[-1]);print('mesh gym',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['config']['kernel_resources'])"
timeout -k 10 400 python3 -u tools/mesh_c3.py 4096 main_mesh > $D/mesh_c3.txt 2>&1 || exit $?
cut -c1-250 $D/mesh_c3.txt
