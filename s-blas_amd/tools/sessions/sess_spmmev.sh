#!/bin/bash
# config-4 SpMM evidence: FETCH/WRITE/L2 passes -> profiles/pmc_spmm_ctile.json, kernel
# trace of the bench command, then the bench line with cpu_baseline and traffic
set -o pipefail
O=gpurun_out/spmm
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
D="s-blas_amd/tools/bench_spmm.py --steps 3 --warmup 1 --no-cpu-baseline"
$T 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $D > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
$T 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $D > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
$T 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o run --output-format csv -- python3 $D > $O/l2.log 2>&1 || { tail -5 $O/l2.log; exit 1; }
python3 s-blas_amd/tools/pmc_traffic.py --kernel k_spmm_ctile,k_spmm_ctreduce --fetch $O/fetch --write $O/write --l2 $O/l2 --algorithmic 699177252 --out profiles/pmc_spmm_ctile.json > /dev/null || exit 1
cat profiles/pmc_spmm_ctile.json | head -20
$T 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -E "k_spmm" $O/prof/run_kernel_stats.csv | cut -c1-160
$T 300 python3 s-blas_amd/tools/bench_spmm.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
