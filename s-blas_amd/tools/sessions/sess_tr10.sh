#!/bin/bash
# transpose + scan users: parity, then per-kernel times for the variants given as env strings
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_spmv_gpu.py -k "transpose or sptrans or csr5 or panel" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for v in "$@"; do
  i=$((i+1))
  env $v $T 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_tr$i -o tr -- python3 $R/s-blas_amd/tools/bench_transpose.py --mgpu= > $R/gpurun_out/prof_tr$i.log 2>&1 || { tail -20 $R/gpurun_out/prof_tr$i.log; exit 1; }
  echo "== $v: $(grep -o '"ms": [0-9.]*' $R/gpurun_out/prof_tr$i.log)"
  python3 $R/s-blas_amd/tools/rocpd_stats.py $(find $R/gpurun_out/prof_tr$i -name '*.db' | head -1) | cut -c1-40,110-160 | head -9
done
