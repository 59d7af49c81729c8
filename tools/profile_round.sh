#!/bin/bash
# Round profile: bench line + rocprofv3 kernel stats + HBM PMC passes (separate runs, no tracing
# domains beside --pmc).  Usage: tools/profile_round.sh OUTDIR [bench args, e.g. --model main_mesh]
# (writes under gpurun_out/OUTDIR)
set -o pipefail
R=$(pwd)
D=$R/gpurun_out/$1
shift
X="$*"
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 bench.py $X > $D/bench.json 2> $D/bench.err || exit $?
tail -1 $D/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $X --steps 50 --warmup 5 --no-cpu-baseline --no-extra > $D/trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $D/pmc_$c -o run -- python3 bench.py $X --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $D/pmc_$c.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $D/pmc_sq -o run -- python3 bench.py $X --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $D/pmc_sq.log 2>&1 || exit $?
# lane utilisation (thread-cycles per VALU cycle) and the FP64 instruction mix
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_WAVES --output-format csv -d $D/pmc_sq2 -o run -- python3 bench.py $X --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $D/pmc_sq2.log 2>&1 || exit $?
python3 tools/filter_csv.py $D/trace/run_kernel_trace.csv $D/pmc_*/run_counter_collection.csv
du -sh $D
