#!/bin/bash
# round 5: pull SpTRSV polls/stores at system scope (sc0 sc1) vs agent (sc1),
# SBLAS_TRSV_SYS experiment, config-5 stand-in -> profiles/r05/trsv_waves/
set -o pipefail
O=gpurun_out/r05_trsv5
mkdir -p $O
T="timeout -k 10 150"
for r in 1 2; do
  for sys in 0 1; do
    SBLAS_TRSV_SYS=$sys $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline > $O/sys${sys}_$r.json 2> $O/sys${sys}_$r.err || { tail -5 $O/sys${sys}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/sys${sys}_$r.json').read().strip().splitlines()[-1]); r=d['executors']
print('sys $sys', {k: (v['ms'], v['rel_l1_vs_xref']) for k, v in r.items() if k in ('pull_csr', 'pull_auto')})"
  done
done
