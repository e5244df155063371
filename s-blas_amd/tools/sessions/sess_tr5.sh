#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for v in "X=1" "SBLAS_TRANSPOSE_WGCU=1" "SBLAS_TRANSPOSE_WGCU=3" "SBLAS_TRANSPOSE_WGCU=4" "SBLAS_TRANSPOSE_MSD_A=6" "SBLAS_TRANSPOSE_MSD_A=8" "SBLAS_TRANSPOSE_MSD_C=8"; do
  env $v $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
  echo "$v $(grep -o "\"ms\": [0-9.]*" gpurun_out/btr.log)"
done
