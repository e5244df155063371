#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "spmm or sptrsv or csrmm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_spmm.log 2>&1 || { tail -30 gpurun_out/t_spmm.log; exit 1; }
tail -1 gpurun_out/t_spmm.log
for p in 0; do
  echo "PIPE=$p"; SBLAS_SPMM_CTPIPE=$p $T 200 python s-blas_amd/tools/bench_spmm.py > gpurun_out/bspmm_p$p.log 2>&1 || { tail -5 gpurun_out/bspmm_p$p.log; exit 1; }
  grep '^{' gpurun_out/bspmm_p$p.log | cut -c1-250
done
$T 300 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 3 --rhs "" > gpurun_out/btrsv.log 2>&1 || { tail -5 gpurun_out/btrsv.log; exit 1; }
grep '^{' gpurun_out/btrsv.log | grep -o '"executors.*' | cut -c1-500
bash s-blas_amd/tools/prof_cmd.sh k_spmm_ctile gpurun_out/pmc_ct0 s-blas_amd/tools/bench_spmm.py --steps 3 --warmup 1 > gpurun_out/pmc_ct0.txt 2>&1 || { tail -5 gpurun_out/pmc_ct0.txt; exit 1; }
cat gpurun_out/pmc_ct0.txt
