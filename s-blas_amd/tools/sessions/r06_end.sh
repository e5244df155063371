# r06 end set (1/2): the default bench line, then rocprofv3 kernel trace + stats
# of the same command (the headline's own rows kept), then FETCH / WRITE / L2
# passes for the headline kernel (xsort) on a headline-only bench command.
set -o pipefail
O=gpurun_out/r06end; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/prof.err || exit 1
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 s-blas_amd/tools/headline_kernels.py "$T" --out $O/headline_kernels.json --rows-out $O/headline_rows.csv > /dev/null || exit 1
S=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
B="bench.py --algo xsort --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-config3 --no-config4 --no-config5 --no-structured --no-rowsplit-beside --no-peak"
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:l2"; do
  C=${pass%%:*}; D=${pass##*:}
  timeout -s KILL 150 rocprofv3 --pmc $C -d $O/xs_$D -o run --output-format csv -- python3 $B > $O/xs_$D.log 2>&1 || exit 1
done
python3 s-blas_amd/tools/pmc_traffic.py --kernel k_spmv_xsort,k_xsort_reduce --fetch $O/xs_fetch --write $O/xs_write --l2 $O/xs_l2 --algorithmic 533000004 --out $O/pmc_xsort.json > /dev/null
