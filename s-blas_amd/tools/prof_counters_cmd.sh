#!/bin/bash
# Counter passes over any python command, one rocprofv3 --pmc run per counter
# group (the hardware's per-block slot limits), each bounded:
#   prof_counters_cmd.sh <kernel-substring> <outdir> <python args...>
# (environment for the run: set it before calling this script)
set -o pipefail
K=$1; O=$2; shift 2
mkdir -p $O
export TMPDIR=/tmp
i=0
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -d $O/p$i -o run --output-format csv -- python3 "$@" > $O/p$i.log 2>&1 || { echo "pass $i ($G) failed"; tail -5 $O/p$i.log; exit 1; }
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES
SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TCC_TAG_STALL_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
GROUPS
python3 s-blas_amd/tools/pmc_summary.py --kernel "$K" --json $O/summary.json $O/p*
