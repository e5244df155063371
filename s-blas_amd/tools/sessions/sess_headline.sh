#!/bin/bash
# Headline evidence for this round: default bench line, rocprofv3 kernel-trace
# stats of the same command, FETCH/WRITE/L2 counter passes -> profiles/pmc_xsort.json
set -o pipefail
O=gpurun_out/hl
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | cut -c1-400
$T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-300
D="s-blas_amd/tools/spmv_one.py --algo xsort --reps 6"
$T 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $D > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
$T 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $D > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
$T 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o run --output-format csv -- python3 $D > $O/l2.log 2>&1 || { tail -5 $O/l2.log; exit 1; }
python3 s-blas_amd/tools/pmc_traffic.py --kernel k_spmv_xsort,k_xsort_reduce --fetch $O/fetch --write $O/write --l2 $O/l2 --algorithmic 533000004 --out $O/pmc_xsort.json || exit 1
cat $O/pmc_xsort.json
