#!/bin/bash
# round 5: slot-parallel C-tile reduce: SpMM tests, slice tables rows / cols /
# grid, N = 8 kernel trace -> profiles/r05/spmm_grid/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_grid4
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread -k "spmm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sp in rows cols grid; do
  $T 300 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1,2,4,8 --reps 8 --split $sp > $O/slices_$sp.jsonl 2> $O/slices_$sp.err || { tail -5 $O/slices_$sp.err; exit 1; }
done
grep -h summary $O/slices_*.jsonl | cut -c1-100
for sp in rows grid; do
  $T 300 rocprofv3 --kernel-trace --stats -d $O/prof_$sp -o run --output-format csv -- python3 s-blas_amd/tools/bench_spmm_slices.py --worlds 8 --reps 4 --split $sp > $O/slices8_$sp.jsonl 2> $O/slices8_$sp.err || { tail -5 $O/slices8_$sp.err; exit 1; }
done
