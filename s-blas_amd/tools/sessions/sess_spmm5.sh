#!/bin/bash
# owned-row C tile: parity (kernel tests + full config 4), timing vs the atomic tile, counters
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "spmm or csrmm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_spmm.log 2>&1 || { tail -30 gpurun_out/t_spmm.log; exit 1; }
tail -1 gpurun_out/t_spmm.log
$T 600 python -u -m pytest tests/test_configs_gpu.py -k "config4" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_cfg4.log 2>&1 || { tail -30 gpurun_out/t_cfg4.log; exit 1; }
tail -1 gpurun_out/t_cfg4.log
for v in "SBLAS_SPMM_CTOWN=1" "SBLAS_SPMM_CTOWN=0"; do
  echo "$v"; env $v $T 200 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > gpurun_out/bspmm.log 2>&1 || { tail -5 gpurun_out/bspmm.log; exit 1; }
  grep '^{' gpurun_out/bspmm.log | cut -c1-300
done
bash s-blas_amd/tools/prof_cmd.sh k_spmm_ctown gpurun_out/pmc_co s-blas_amd/tools/bench_spmm.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_co.txt 2>&1 || { tail -5 gpurun_out/pmc_co.txt; exit 1; }
grep -E "LDS|TD_|TA_TA|VALU|TCC_HIT|TCC_MISS|GRBM_GUI" gpurun_out/pmc_co.txt
