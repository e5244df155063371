# round-3 end evidence (profiles/r03/end/): FETCH/WRITE/L2 counter passes of the
# bench command -> pmc_xsort.json, the default bench line, rocprofv3 kernel-trace
# stats of that same command, prefix-column lines, the full -m gpu suite, smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_end
mkdir -p $O
T="timeout -k 10"
P="bench.py --no-cpu-baseline --no-rowsplit-beside --steps 5 --warmup 2"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $P > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $P > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o run --output-format csv -- python3 $P > $O/l2.log 2>&1 || { tail -5 $O/l2.log; exit 1; }
python3 s-blas_amd/tools/pmc_traffic.py --kernel k_spmv_xsort,k_xsort_reduce --fetch $O/fetch --write $O/write --l2 $O/l2 --algorithmic 533000004 --out $O/pmc_xsort.json || exit 1
cp $O/pmc_xsort.json profiles/pmc_xsort.json
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
$T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
for a in rowsplit csr5 xsort; do
  $T 300 python bench.py --cols prefix --algo $a --no-cpu-baseline > $O/bench_prefix_$a.json 2> $O/prefix_$a.err || { tail -20 $O/prefix_$a.err; exit 1; }
done
$T 1500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo done
