#!/bin/bash
# round 5: poll back-off of the natural-order pull at the 2-waves-per-CU
# default (SBLAS_TRSV_SLEEP fixed 1 / 2 / 4, adaptive -2 / -4 / -6), and 3
# waves per CU with adaptive back-off, on the config-5 stand-in -> profiles/r05/trsvsleep/
set -o pipefail
O=gpurun_out/r05_trsvsleep
mkdir -p $O
T="timeout -k 10 150"
for r in 1 2; do
for c in "1 128" "2 128" "4 128" "-2 128" "-4 128" "-6 128" "-4 192" "-6 256"; do
  set -- $c
  SBLAS_TRSV_SLEEP=$1 SBLAS_TRSV_THREADS=$2 $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline > $O/s$1_t$2_$r.json 2> $O/s$1_t$2_$r.err || { tail -5 $O/s$1_t$2_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/s$1_t$2_$r.json').read().strip().splitlines()[-1]); r=d['executors']
print('sleep $1 threads $2', r['pull_csr']['ms'])"
done
done
