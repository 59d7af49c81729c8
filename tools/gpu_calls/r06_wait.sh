#!/bin/bash
# round-6 GPU call: where the waves of the headline kernel wait at the round-6 head (LDS / VMEM latency,
# instruction mix, active and wait cycles, L1 traffic; one rocprofv3 --pmc pass per group) -> gpurun_out/$1
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
B="python3 bench.py --steps 10 --warmup 2 --pre-steps 100 --no-cpu-baseline --no-extra ${X:-}"
i=0
for P in "LdsLatency" "VmemLatency" \
         "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_FLAT" \
         "SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" \
         "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM_NORM SQ_INST_CYCLES_SMEM SQ_WAVE_CYCLES" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $D/p$i -o run -- $B > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
done
python3 tools/pmc_breakdown.py $D > /dev/null && echo breakdown ok
