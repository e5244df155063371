#!/bin/bash
# round 5: pull SpTRSV with fewer spinning waves (SBLAS_TRSV_THREADS 64 / 128
# per workgroup, one workgroup per CU; and 2 / CU at 64) on the config-5
# stand-in -> profiles/r05/trsv_waves/
set -o pipefail
O=gpurun_out/r05_trsv
mkdir -p $O
T="timeout -k 10 150"
for c in "256 1" "128 1" "64 1" "64 2" "256 1"; do
  set -- $c
  SBLAS_TRSV_THREADS=$1 SBLAS_TRSV_WG_PER_CU=$2 $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline > $O/t$1_w$2.json 2> $O/t$1_w$2.err || { tail -5 $O/t$1_w$2.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/t$1_w$2.json').read().strip().splitlines()[-1]); r=d['executors']
print('threads $1 per_cu $2', {k: (v['ms'], v['rel_l1_vs_xref']) for k, v in r.items() if isinstance(v, dict) and 'ms' in v and k.startswith('pull')})"
done
