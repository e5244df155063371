#!/bin/bash
# xsort planner with binary-search range cuts: parity, then plan-build time and kernel A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py tests/test_ctx_gpu.py -m gpu -x -q -k "xsort or 5 or config2_full" --timeout 300 --timeout-method thread > gpurun_out/plan_tests.log 2>&1 || { tail -30 gpurun_out/plan_tests.log; exit 1; }
tail -1 gpurun_out/plan_tests.log
bash s-blas_amd/tools/exp_ab.sh 2>&1 | tee gpurun_out/plan_ab.txt
SBLAS_XS_TIMING=1 timeout -k 10 120 python3 s-blas_amd/tools/spmv_one.py --reps 3 2>&1 | grep -E "xsort" | tee gpurun_out/plan_phases.txt
