#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for L in "" s-blas_amd/ab/libsblas_r2t256.so; do
 for a in msd lsd; do
  env ${L:+SBLAS_LIB=$L} SBLAS_TRANSPOSE_ALGO=$a $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
  echo "lib=$L algo=$a $(grep -o "\"ms\": [0-9.]*" gpurun_out/btr.log)"
 done
done
