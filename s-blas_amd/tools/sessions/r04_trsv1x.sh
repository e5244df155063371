#!/bin/bash
# round 4: SpTRSV pull on ONE XCD (SBLAS_TRSV_ONEXCD=1: every dependency hop within one L2)
# vs the whole chip, config 5 stand-in; 1 / 2 / 4 workgroups per CU
set -o pipefail
O=gpurun_out/r04_trsv1x; mkdir -p $O
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 5 > $O/$tag.json 2>>$O/err.log || { echo "$tag failed"; tail -5 $O/err.log; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); e=d['executors']
print('$tag', {k:(v['ms'], '%.1e' % v['rel_l1_vs_xref']) for k,v in e.items() if k!='push_csc'})"
}
run chip X=1 && run one SBLAS_TRSV_ONEXCD=1 && run one_wg2 SBLAS_TRSV_ONEXCD=1 SBLAS_TRSV_WG_PER_CU=2 \
  && run one_wg4 SBLAS_TRSV_ONEXCD=1 SBLAS_TRSV_WG_PER_CU=4
