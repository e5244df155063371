#!/bin/bash
# round-end evidence after the plan-build changes: SpMM config-4 line (plan time), then
# the full suite, smoke, default bench line and rocprofv3 stats (sess_r2end.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 s-blas_amd/tools/bench_spmm.py > gpurun_out/bench_spmm_cfg4.json 2> gpurun_out/bench_spmm.err || { tail -20 gpurun_out/bench_spmm.err; exit 1; }
cat gpurun_out/bench_spmm_cfg4.json
bash s-blas_amd/tools/sessions/sess_r2end.sh
