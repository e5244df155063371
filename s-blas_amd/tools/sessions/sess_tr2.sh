#!/bin/bash
# MSD transpose: parity (transpose, sptrsv which builds CSR by transposing, CLI), timing vs LSD, kernel stats
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cli_gpu.py -k "transpose or sptrans or sptrsv or sptrsm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
$T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
grep '^{' gpurun_out/btr.log | cut -c1-400
SBLAS_TRANSPOSE_ALGO=lsd $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr_lsd.log 2>&1 || { tail -5 gpurun_out/btr_lsd.log; exit 1; }
grep '^{' gpurun_out/btr_lsd.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && $T 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/s-blas_amd/tools/bench_transpose.py --mgpu= > $GRAFT_REPO_ROOT/gpurun_out/prof_tr.log 2>&1 || exit 1
cat $(find $GRAFT_REPO_ROOT/gpurun_out/prof_tr -name "*kernel_stats.csv") | cut -c1-160 | head -20
