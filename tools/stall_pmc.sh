#!/bin/bash
# Where the queue kernel's wave-cycles go (round 3): two SQ passes on the bench workload, one counter
# set each (rocprofv3 does not split passes): issue/active/wait buckets (disjoint: WAIT_ANY +
# WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, quad-cycles) with the GRBM clock, then the
# per-pipe active cycles.  tools/stall_summary.py turns them into per-wave shares.
# usage: tools/stall_pmc.sh OUTDIR [extra bench args]
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; shift; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
P3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_CYCLES"
# latency per memory instruction type (INST_LEVEL = outstanding instructions summed per cycle) and
# the instruction cache (the queue kernel is ~46k instructions)
P4="SQ_WAVES SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_IFETCH"
P5="SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH_LEVEL"
PASSES=${PASSES:-"1 2 3 4 5"}
for i in $PASSES; do
  eval P=\$P$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $D/p$i -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-extra "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
done
python3 tools/filter_csv.py $D/p*/run_counter_collection.csv > /dev/null; python3 tools/stall_summary.py $D > $D/stall.json && cat $D/stall.json
