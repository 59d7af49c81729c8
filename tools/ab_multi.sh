#!/bin/bash
# Same-box A/B/C...: the product library against variants built ON THE BOX from patches against HEAD
# (tools/var/<name>.patch) and/or extra compiler flags (tools/var/<name>.flags), so no variant
# library rides in the push.  Each variant first runs the fast
# GPU parity set; then the bench alternates base and variants for ROUNDS rounds (boxes differ by ~1 %).
# usage: tools/ab_multi.sh ROUNDS NAME...   (AB_EXTRA=1: the bench's other configs too, printed beside)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/ab; mkdir -p $D
ROUNDS=$1; shift
FL="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -disable-machine-licm -Wno-unused-result"
pids=""
for v in "$@"; do
  W=/tmp/ur3e_var_$v; rm -rf $W; mkdir -p $W; cp -r $R/ur3e_amd $R/include $W/
  if [ -f $R/tools/var/$v.patch ]; then (cd $W && patch -s -p1 < $R/tools/var/$v.patch) || { echo "patch $v failed"; exit 1; }; fi
  XF=""; if [ -f $R/tools/var/$v.flags ]; then XF=$(cat $R/tools/var/$v.flags); fi
  timeout -k 10 600 /opt/rocm/bin/hipcc $FL $XF -o $W/lib.so $W/ur3e_amd/csrc/ur3e_batch.hip $W/ur3e_amd/csrc/ur3e_vecnorm.hip $W/ur3e_amd/csrc/ur3e_mjcf.cpp $W/ur3e_amd/csrc/ur3e_gather.cpp -ldl > $D/${v}_build.log 2>&1 &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "a variant build failed"; tail -5 $D/*_build.log; exit 1; }; done
for v in "$@"; do
  UR3E_LIB=/tmp/ur3e_var_$v/lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py -x -q --timeout 200 --timeout-method thread -k "not 1000 and not trace and not occupancy" > $D/${v}_parity.txt 2>&1 || { echo "$v parity FAILED"; tail -30 $D/${v}_parity.txt; exit 1; }
  echo "$v parity: $(tail -1 $D/${v}_parity.txt)"
done
for i in $(seq 1 $ROUNDS); do
  for v in base "$@"; do
    if [ $v = base ]; then unset UR3E_LIB; else export UR3E_LIB=/tmp/ur3e_var_$v/lib.so; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline ${AB_EXTRA:+} $( [ -n "$AB_EXTRA" ] || echo --no-extra ) > $D/$v$i.json 2> $D/$v$i.err || { echo "$v failed"; tail -3 $D/$v$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$v$i.json').read().strip().splitlines()[-1]);x=d.get('other_configs') or {};print('$v',round(d['value']/1e6,4),round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), *[(k[:14], round(v['value']/1e6,3)) for k,v in x.items() if isinstance(v,dict) and 'value' in v])"
  done
done
unset UR3E_LIB
