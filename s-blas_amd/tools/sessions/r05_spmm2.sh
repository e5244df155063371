#!/bin/bash
# round 5: C-tile SpMM with two 64-entry steps per wave iteration
# (SBLAS_SPMM_CTU=2) on configs[3]: parity, cold kernel times (alternating),
# counters -> profiles/r05/spmm_u2/
set -o pipefail
O=gpurun_out/r05_spmm2
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -k "spmm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  $T 200 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 8 > $O/def$r.jsonl 2>&1 || exit 1
  SBLAS_SPMM_CTU=2 $T 200 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 8 > $O/u2_$r.jsonl 2>&1 || exit 1
done
grep -h summary $O/def*.jsonl $O/u2_*.jsonl
SBLAS_SPMM_CTU=2 bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmm_ctile" $O/pmc_u2 s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 2 || exit 1
