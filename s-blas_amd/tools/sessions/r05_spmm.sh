#!/bin/bash
# round 5: scalar-prefetch microbenchmark (tools/exp/spf.hip) and the C-tile
# SpMM's software-pipelined stream loads (SBLAS_SPMM_CTPIPE) on configs[3]:
# parity, cold kernel times (alternating), counters -> profiles/r05/spmm_pipe/
set -o pipefail
O=gpurun_out/r05_spmm
mkdir -p $O
T="timeout -k 10"
$T 120 s-blas_amd/tools/exp_spf > $O/spf.jsonl 2>&1 || exit 1
$T 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -k "spmm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  $T 200 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 8 > $O/def$r.jsonl 2>&1 || exit 1
  SBLAS_SPMM_CTPIPE=1 $T 200 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 8 > $O/pipe$r.jsonl 2>&1 || exit 1
done
grep -h summary $O/def*.jsonl $O/pipe*.jsonl
bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmm_ctile" $O/pmc_def s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 2 || exit 1
SBLAS_SPMM_CTPIPE=1 bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmm_ctile" $O/pmc_pipe s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 2 || exit 1
