#!/bin/bash
set -o pipefail
bash s-blas_amd/tools/prof_cmd.sh k_rx2_scatter gpurun_out/pmc_tr s-blas_amd/tools/bench_transpose.py --mgpu= --steps 4 > gpurun_out/pmc_tr.txt 2>&1 || { tail -5 gpurun_out/pmc_tr.txt; exit 1; }
cat gpurun_out/pmc_tr.txt
