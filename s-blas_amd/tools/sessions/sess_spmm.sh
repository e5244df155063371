#!/bin/bash
# round-2 session: SpMM C-tile + level-set SpTRSV tests, then their benchmarks
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "spmm or sptrsv or csrmm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_spmm.log 2>&1 || { tail -30 gpurun_out/t_spmm.log; exit 1; }
tail -2 gpurun_out/t_spmm.log
$T 400 python -u -m pytest tests/test_cli_gpu.py -k "spmm_two_ranks" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_2r.log 2>&1 || { tail -30 gpurun_out/t_2r.log; exit 1; }
$T 400 python -u -m pytest tests/test_configs_gpu.py -k "config4 or config5_single" -x -q --timeout 250 --timeout-method thread > gpurun_out/t_cfg4.log 2>&1 || { tail -30 gpurun_out/t_cfg4.log; exit 1; }
tail -2 gpurun_out/t_cfg4.log
for w in 11 10 12 9; do
  echo "CTW=$w"; SBLAS_SPMM_CTW=$w $T 200 python s-blas_amd/tools/bench_spmm.py > gpurun_out/bspmm_ct$w.log 2>&1 || { tail -5 gpurun_out/bspmm_ct$w.log; exit 1; }
  cut -c1-330 gpurun_out/bspmm_ct$w.log
done
echo "l2slice"; SBLAS_SPMM_CTILE=0 $T 200 python s-blas_amd/tools/bench_spmm.py > gpurun_out/bspmm_l2.log 2>&1 && cut -c1-330 gpurun_out/bspmm_l2.log
$T 300 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 3 > gpurun_out/btrsv.log 2>&1 || { tail -5 gpurun_out/btrsv.log; exit 1; }
cut -c1-900 gpurun_out/btrsv.log
