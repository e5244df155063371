#!/bin/bash
set -o pipefail
T="timeout -k 10 200"
for v in "SBLAS_SPMM_CTR=1204" "SBLAS_SPMM_CTR=600 SBLAS_SPMM_CTNS=1" "SBLAS_SPMM_CTR=600 SBLAS_SPMM_CTNS=2" "SBLAS_SPMM_CTR=400 SBLAS_SPMM_CTNS=1" "SBLAS_SPMM_CTR=800 SBLAS_SPMM_CTNS=1"; do
  echo -n "$v: "; env $v $T python s-blas_amd/tools/bench_spmm.py 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernel_ms_max_over_ranks'])" || exit 1
done
