#!/bin/bash
# SpMM plan build with the block analysis in parallel: parity (SpMM tests incl. MFMA tiles and config 4), then the config-4 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "spmm or csrmm or config4" --timeout 300 --timeout-method thread > gpurun_out/spmm_plan_tests.log 2>&1 || { tail -30 gpurun_out/spmm_plan_tests.log; exit 1; }
tail -1 gpurun_out/spmm_plan_tests.log
timeout -k 10 300 python3 s-blas_amd/tools/bench_spmm.py > gpurun_out/bench_spmm_cfg4.json 2> gpurun_out/bench_spmm.err || { tail -20 gpurun_out/bench_spmm.err; exit 1; }
cat gpurun_out/bench_spmm_cfg4.json
