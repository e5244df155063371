#!/bin/bash
set -o pipefail
O=gpurun_out/hl2
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_spmv_gpu.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
$T 400 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | cut -c1-330
$T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
grep -E "k_spmv_xsort|k_xsort_reduce" $O/prof/run_kernel_stats.csv | cut -d, -f1-5 | sed 's/(sblas::Xs[^"]*//;s/(sblas::XsRange[^"]*//'
