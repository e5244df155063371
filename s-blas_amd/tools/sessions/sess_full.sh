#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in "SBLAS_SPMM_CTPAIR=1" "SBLAS_SPMM_CTPAIR=0"; do
  echo "$v"; env $v $T 200 python s-blas_amd/tools/bench_spmm.py > gpurun_out/bspmm.log 2>&1 || { tail -5 gpurun_out/bspmm.log; exit 1; }
  grep '^{' gpurun_out/bspmm.log | cut -c1-250
done
