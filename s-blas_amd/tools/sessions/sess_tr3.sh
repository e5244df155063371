#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "transpose or sptrsv_kat or sptrans" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
for c in 7 8 6; do
  SBLAS_TRANSPOSE_MSD_C=$c $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
  echo "MSD_C=$c $(grep '^{' gpurun_out/btr.log | cut -c1-200)"
done
cd /tmp && export TMPDIR=/tmp && $T 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/s-blas_amd/tools/bench_transpose.py --mgpu= > $GRAFT_REPO_ROOT/gpurun_out/prof_tr.log 2>&1 || exit 1
