#!/bin/bash
# Per-stage VALU instruction classes of the compact tier (round 3): builds the -DUR3E_DOUBLE_STAGE=k
# variants ON THE BOX (into gpurun_out, so they never ride in the push), then one 8-counter SQ pass
# per variant (F64 add/mul/fma/trans, int32, all VALU, SALU, waves) on the bench workload.
# tools/stage_insts.py turns the deltas against the product build into per-stage classes.
# usage: tools/stage_classes.sh OUTDIR
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; L=$D/libs; mkdir -p $L
cd /tmp && export TMPDIR=/tmp && cd $R
FL="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -disable-machine-licm -Wno-unused-result"
SRC="ur3e_amd/csrc/ur3e_batch.hip ur3e_amd/csrc/ur3e_vecnorm.hip"
VS="0 4 5 6 7 8 15 20 21 22 23"
pids=""
for k in $VS; do
  timeout -k 10 600 /opt/rocm/bin/hipcc $FL -DUR3E_DOUBLE_STAGE=$k -o $L/dbl$k.so $SRC > $L/dbl$k.log 2>&1 &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "a variant build failed"; tail -5 $L/*.log; exit 1; }; done
echo "built: $(ls $L/*.so | wc -l) variants"
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU"
for v in base $(for k in $VS; do echo dbl$k; done); do
  if [ $v = base ]; then unset UR3E_LIB; else export UR3E_LIB=$L/$v.so; fi
  timeout -k 10 120 rocprofv3 --pmc $CNT --output-format csv -d $D/$v -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-extra > $D/$v.log 2>&1 || { echo "$v failed"; tail -5 $D/$v.log; exit 1; }
  echo "$v done"
done
unset UR3E_LIB
python3 tools/filter_csv.py $D/*/run_counter_collection.csv > /dev/null
rm -rf $L
python3 tools/stage_insts.py $D > $D/stage_classes.json && tail -5 $D/stage_classes.json
