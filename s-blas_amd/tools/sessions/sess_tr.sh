#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "transpose or sptrans or sptrsv" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
$T 300 python s-blas_amd/tools/bench_transpose.py > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
grep '^{' gpurun_out/btr.log | cut -c1-600
SBLAS_TRANSPOSE_WGCU=4 $T 300 python s-blas_amd/tools/bench_transpose.py > gpurun_out/btr8.log 2>&1 || { tail -5 gpurun_out/btr8.log; exit 1; }
grep '^{' gpurun_out/btr8.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && $T 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/s-blas_amd/tools/bench_transpose.py > $GRAFT_REPO_ROOT/gpurun_out/prof_tr.log 2>&1 || exit 1
cat $(find $GRAFT_REPO_ROOT/gpurun_out/prof_tr -name "*kernel_stats.csv") | cut -c1-200 | head -20
