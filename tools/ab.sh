#!/bin/bash
# A/B on one GPU box: the product library against ur3e_amd/_lib/libur3e_amd_var.so, alternating runs
# (boxes differ by ~1 %, so variants are compared within one call).  usage: [AB_ARGS='--model main_mesh'] tools/ab.sh [rounds]
set -o pipefail
D=gpurun_out/ab${AB_TAG:-}; mkdir -p $D
for i in $(seq 1 ${1:-3}); do
  for v in base var; do
    if [ $v = base ]; then unset UR3E_LIB; else export UR3E_LIB=$PWD/ur3e_amd/_lib/libur3e_amd_var.so; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra ${AB_ARGS:-} > $D/$v$i.json 2> $D/$v$i.err || { echo "$v failed"; tail -3 $D/$v$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$v$i.json').read().strip().splitlines()[-1]);print('$v',round(d['value']/1e6,4),round(d['ms_per_step'],4))"
  done
done
