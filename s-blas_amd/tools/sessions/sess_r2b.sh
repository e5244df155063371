#!/bin/bash
# round-2 session b: C-tile v2 SpMM + grid-barrier level-set tests and benches
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "spmm or sptrsv or csrmm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_spmm.log 2>&1 || { tail -30 gpurun_out/t_spmm.log; exit 1; }
tail -2 gpurun_out/t_spmm.log
for w in 11 9; do
  echo "CTW=$w"; SBLAS_SPMM_CTW=$w $T 200 python s-blas_amd/tools/bench_spmm.py > gpurun_out/bspmm_ct$w.log 2>&1 || { tail -5 gpurun_out/bspmm_ct$w.log; exit 1; }
  cut -c1-330 gpurun_out/bspmm_ct$w.log | grep '^{'
done
$T 300 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 3 --rhs "" > gpurun_out/btrsv.log 2>&1 || { tail -5 gpurun_out/btrsv.log; exit 1; }
grep '^{' gpurun_out/btrsv.log | cut -c1-900
