#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_spmv_gpu.py -k "xsort" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_xs.log 2>&1 || { tail -30 gpurun_out/t_xs.log; exit 1; }
tail -1 gpurun_out/t_xs.log
$T 600 python -u -m pytest tests/test_configs_gpu.py -k "config2_full_size and xsort" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_cfg2xs.log 2>&1 || { tail -30 gpurun_out/t_cfg2xs.log; exit 1; }
tail -1 gpurun_out/t_cfg2xs.log
R="$T 90 python3 s-blas_amd/tools/spmv_one.py --reps 30 --cold --scrub read"
for i in 1 2; do
  echo -n "k24 u1: "; $R 2>/dev/null | tail -1 || exit 1
  echo -n "k24 u2: "; SBLAS_XS_U=2 $R 2>/dev/null | tail -1 || exit 1
  echo -n "k32:    "; SBLAS_XS_K24=0 $R 2>/dev/null | tail -1 || exit 1
done
