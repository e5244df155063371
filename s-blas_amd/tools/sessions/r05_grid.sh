#!/bin/bash
# round 5: SpMM 2-D grid split (sblas_dist.spmm_grid_shape) and the C tile's
# slab sets sized by the call's column groups: SpMM tests, per-rank slice
# tables for rows / cols / grid at N = 1, 2, 4, 8 -> profiles/r05/spmm_grid/
set -o pipefail
O=gpurun_out/r05_grid
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread -k "spmm or config3_two_ranks" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sp in rows cols grid; do
  $T 300 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1,2,4,8 --reps 8 --split $sp > $O/slices_$sp.jsonl 2> $O/slices_$sp.err || { tail -5 $O/slices_$sp.err; exit 1; }
done
grep -h summary $O/slices_*.jsonl
