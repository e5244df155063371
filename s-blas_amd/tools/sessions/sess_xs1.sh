#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
rm -f gpurun_out/xs_trace.txt
SBLAS_XS_TRACE=gpurun_out/xs_trace.txt $T 120 python3 s-blas_amd/tools/spmv_one.py --algo xsort --reps 4 --cold --scrub read > gpurun_out/xs_trace_run.log 2>&1 || { tail -5 gpurun_out/xs_trace_run.log; exit 1; }
python3 s-blas_amd/tools/xs_trace.py gpurun_out/xs_trace.txt
$T 120 python3 s-blas_amd/tools/spmv_one.py --algo xsort --reps 20 --cold --scrub read
bash s-blas_amd/tools/prof_cmd.sh k_spmv_xsort gpurun_out/pmc_xs s-blas_amd/tools/spmv_one.py --algo xsort --reps 6 > gpurun_out/pmc_xs.txt 2>&1 || { tail -5 gpurun_out/pmc_xs.txt; exit 1; }
cat gpurun_out/pmc_xs.txt
