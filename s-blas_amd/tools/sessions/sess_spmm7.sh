#!/bin/bash
# SpMM: the product build against a timing-experiment build (SBLAS_LIB), alternating
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for r in 1 2; do
for L in "" "s-blas_amd/ab/libsblas_exp.so"; do
  SBLAS_LIB=$L $T 200 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > gpurun_out/bspmm.log 2>&1 || { tail -5 gpurun_out/bspmm.log; exit 1; }
  echo "lib=${L:-product} $(grep -o '"kernel_ms_max_over_ranks": [0-9.]*' gpurun_out/bspmm.log)"
done
done
