#!/bin/bash
# rocprofv3 kernel-trace stats + PMC traffic for the column-sorted SpMV on the
# config-2 matrix (one pass per counter group, each under its own timeout).
set -o pipefail
O=gpurun_out/pxs; mkdir -p $O
export TMPDIR=/tmp
V="$1"   # optional env assignments, e.g. "SBLAS_XS_ROWS=8192"
B="bench.py --algo xsort --no-cpu-baseline --steps 5 --warmup 1"
env $V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $B > $O/trace.log 2>&1 || exit 1
env $V timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python $B > $O/fetch.log 2>&1 || exit 1
env $V timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python $B > $O/write.log 2>&1 || exit 1
env $V timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o run --output-format csv -- python $B > $O/l2.log 2>&1 || exit 1
python3 s-blas_amd/tools/pmc_traffic.py --kernel k_spmv_xsort,k_xsort_reduce --fetch $O/fetch --write $O/write --l2 $O/l2 --algorithmic 533000004 --out $O/pmc_xsort.json > /dev/null || exit 1
cat $O/pmc_xsort.json
f=$(find $O/trace -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -12
