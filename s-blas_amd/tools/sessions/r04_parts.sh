#!/bin/bash
# round 4: kernel cost of the overlapped exchange's parts (rank-0 slices cut into K parts)
set -o pipefail
O=gpurun_out/r04_parts; mkdir -p $O
for K in 2 4; do
  timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort,panel --parts $K > $O/slice_parts$K.jsonl 2>>$O/err.log || exit 1
done
for K in 2 4; do
  timeout -k 10 200 python bench.py --driver ctx --overlap $K --no-config3 --no-cpu-baseline > $O/bench_ctx1_overlap$K.json 2>>$O/err.log || exit 1
done
cat $O/slice_parts*.jsonl | cut -c1-400
