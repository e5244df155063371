#!/bin/bash
# does x arriving warm change the slice's cold span? (N = 1 and 8, xsort)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 200"
$T python3 s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort --reps 10 || exit 1
$T python3 s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort --reps 10 --warm-x || exit 1
