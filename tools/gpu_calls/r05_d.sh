#!/bin/bash
# round-5 GPU call: the GPU suite, the mesh model's profile (trace + PMC), gym tiers of both compiles,
# the full bench line (C3 mesh, C5 legs)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.txt 2>&1 || { tail -40 $D/gpu_tests.txt; exit 1; }
tail -2 $D/gpu_tests.txt
timeout -k 10 300 python3 -u tools/gym_tiers.py 4096 600 100 main_mesh > $D/gym_tiers_mesh.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gym_tiers.py 4096 600 100 main > $D/gym_tiers_main.txt 2>&1 || exit $?
cut -c1-220 $D/gym_tiers_mesh.txt $D/gym_tiers_main.txt
bash tools/profile_round.sh $1/mesh_prof --model main_mesh || exit $?
timeout -k 10 900 python3 bench.py > $D/bench.json 2> $D/bench.err || exit $?
python3 -c "import json;d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]);print(d['value']);x=d['other_configs'];print(json.dumps({k:(v.get('value') if isinstance(v,dict) else v) for k,v in x.items()}));print(json.dumps(x.get('C5_ppo_rollout'))[:600]);print(json.dumps(x.get('C3_main_mesh_move_l_mug'))[:600])"
