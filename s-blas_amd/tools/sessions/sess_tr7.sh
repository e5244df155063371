#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "transpose" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
for v in "SBLAS_TRANSPOSE_DIRECT=0" "SBLAS_TRANSPOSE_DIRECT=1" "SBLAS_TRANSPOSE_DIRECT=0" "SBLAS_TRANSPOSE_DIRECT=1"; do
  env $v $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/btr.log)"
done
