#!/bin/bash
# transpose: parity, A/B timing against the previous build, kernel stats
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -k "transpose or sptrans" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
for i in 1 2; do
  $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr.log 2>&1 || { tail -5 gpurun_out/btr.log; exit 1; }
  echo "new  $(grep -o '"ms": [0-9.]*' gpurun_out/btr.log)"
  SBLAS_LIB=s-blas_amd/ab/libsblas_prev.so $T 300 python s-blas_amd/tools/bench_transpose.py --mgpu= > gpurun_out/btr_prev.log 2>&1 || { tail -5 gpurun_out/btr_prev.log; exit 1; }
  echo "prev $(grep -o '"ms": [0-9.]*' gpurun_out/btr_prev.log)"
done
cp gpurun_out/btr.log gpurun_out/bench_transpose.json
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tr -o tr -- python3 $GRAFT_REPO_ROOT/s-blas_amd/tools/bench_transpose.py --mgpu= > $GRAFT_REPO_ROOT/gpurun_out/prof_tr.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_tr.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_tr -name '*kernel_stats.csv' | head -1)
cut -c1-160 "$f" | head -14
