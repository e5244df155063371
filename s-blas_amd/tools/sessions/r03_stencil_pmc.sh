# stencil27 with xsort: L2->fabric bytes (FETCH/WRITE, separate passes) and the
# rocprofv3 kernel trace of the same bench command, to back its 0.84 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_stencil_pmc
mkdir -p $O
P="bench.py --matrix stencil27 --algo xsort --no-cpu-baseline --no-rowsplit-beside --steps 5 --warmup 2"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $P > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $P > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o run --output-format csv -- python3 $P > $O/l2.log 2>&1 || { tail -5 $O/l2.log; exit 1; }
python3 s-blas_amd/tools/pmc_traffic.py --kernel k_spmv_xsort --fetch $O/fetch --write $O/write --l2 $O/l2 --algorithmic 1425272228 --out $O/pmc_stencil27_xsort.json || exit 1
cat $O/pmc_stencil27_xsort.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $P > $O/bench_under_rocprof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cat $O/bench_under_rocprof.json
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -5
echo done
