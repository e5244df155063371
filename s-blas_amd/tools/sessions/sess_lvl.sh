#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "sptrsv" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lvl.log 2>&1 || { tail -30 gpurun_out/t_lvl.log; exit 1; }
tail -1 gpurun_out/t_lvl.log
$T 600 python -u -m pytest tests/test_configs_gpu.py -k "config5_single" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_lvl5.log 2>&1 || { tail -30 gpurun_out/t_lvl5.log; exit 1; }
tail -1 gpurun_out/t_lvl5.log
$T 300 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 3 --rhs "" > gpurun_out/btrsv.log 2>&1 || { tail -5 gpurun_out/btrsv.log; exit 1; }
grep '^{' gpurun_out/btrsv.log | grep -o '"executors.*' | cut -c1-400
