#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -k "spmm or csrmm or config4" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_spmm.log 2>&1 || { tail -30 gpurun_out/t_spmm.log; exit 1; }
tail -1 gpurun_out/t_spmm.log
for r in 1 2 3; do
for v in "SBLAS_SPMM_CTPF=1" "SBLAS_SPMM_CTPF=0"; do
  env $v $T 200 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > gpurun_out/bspmm.log 2>&1 || { tail -5 gpurun_out/bspmm.log; exit 1; }
  echo "$v $(grep -o '"kernel_ms_max_over_ranks": [0-9.]*' gpurun_out/bspmm.log)"
done
done
