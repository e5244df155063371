#!/bin/bash
# round 5: C-tile grid of two workgroups per CU when two tiles fit the LDS
# (rank slices): SpMM tests, slice tables rows / grid -> profiles/r05/spmm_grid/
set -o pipefail
O=gpurun_out/r05_grid2
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "spmm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sp in rows grid; do
  $T 300 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1,2,4,8 --reps 8 --split $sp > $O/slices_$sp.jsonl 2> $O/slices_$sp.err || { tail -5 $O/slices_$sp.err; exit 1; }
done
grep -h summary $O/slices_*.jsonl
