#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 120"
B="python3 s-blas_amd/tools/bench_slice.py --worlds 8 --reps 10"
for p in 4 8 16; do echo "PANELS=$p"; SBLAS_PANELS=$p $T $B --algos panel || exit 1; done
for p in 8 16; do echo "PANELS=$p world 4"; SBLAS_PANELS=$p $T python3 s-blas_amd/tools/bench_slice.py --worlds 4 --reps 10 --algos panel || exit 1; done
