# counters of the default paired layout vs solo light items (SBLAS_XS_SOLO=1):
# L1->L2 read requests, their latency, TCP pending stalls, TA, L2 busy
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_solo_pmc
mkdir -p $O
D="s-blas_amd/tools/spmv_one.py --algo xsort --reps 6"
for mode in base solo; do
  E="SBLAS_XS_SOLO=0"; [ $mode = solo ] && E="SBLAS_XS_SOLO=1"
  i=0; mkdir -p $O/$mode
  while read -r G; do
    [ -z "$G" ] && continue
    i=$((i+1))
    env $E timeout -s KILL 120 rocprofv3 --pmc $G -d $O/$mode/p$i -o run --output-format csv -- python3 $D > $O/$mode/p$i.log 2>&1 || { echo "$mode pass $i ($G) failed"; tail -5 $O/$mode/p$i.log; exit 1; }
  done <<'GROUPS'
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TCC_TAG_STALL_sum
TA_BUSY_max TA_BUSY_min
GROUPS
  python3 s-blas_amd/tools/pmc_summary.py --kernel k_spmv_xsort --json $O/$mode/summary.json $O/$mode/p* > $O/$mode/summary.txt || exit 1
  echo "== $mode"; cat $O/$mode/summary.txt
done
echo done
