#!/bin/bash
# round-5 GPU call: GJK separating-axis early exit in the wave path -- mesh parity, mid-episode stage
# timing and gym tiers of the mesh compile, mesh bench line
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mesh_main.py tests/test_gpu_mesh_c3.py tests/test_gpu_mesh.py -x -q --timeout 500 --timeout-method thread > $D/mesh_tests.txt 2>&1 || { tail -40 $D/mesh_tests.txt; exit 1; }
tail -1 $D/mesh_tests.txt
UR3E_STAGE_MODEL=main_mesh UR3E_STAGE_PRE=500 timeout -k 10 300 python3 -u tools/stage_timing.py 4096 0 gym 0 > $D/stage_main_mesh_pre500.txt 2>&1 || exit $?
grep -E "^(39|48|49|total)" $D/stage_main_mesh_pre500.txt
timeout -k 10 300 python3 -u tools/gym_tiers.py 4096 600 100 main_mesh > $D/gym_tiers_mesh.txt 2>&1 || exit $?
cut -c1-120 $D/gym_tiers_mesh.txt
timeout -k 10 300 python3 bench.py --model main_mesh > $D/bench_mesh.json 2> $D/bench_mesh.err || exit $?
python3 -c "import json;d=json.loads(open('$D/bench_mesh.json').read().strip().splitlines()[-1]);print('mesh gym',d['value'],d['roofline']['kernel_ms'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra > $D/bench_main.json 2> $D/bench_main.err || exit $?
python3 -c "import json;d=json.loads(open('$D/bench_main.json').read().strip().splitlines()[-1]);print('main gym',d['value'],d['roofline']['kernel_ms'])"
timeout -k 10 120 python3 -u tools/vecnorm_trace.py 4096 64 > $D/vecnorm.txt 2>&1 || exit $?
cat $D/vecnorm.txt | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/vn_trace -o run -- python3 tools/vecnorm_trace.py 4096 64 > $D/vn_trace.log 2>&1 || exit $?
head -8 $D/vn_trace/run_kernel_stats.csv | cut -c1-200
