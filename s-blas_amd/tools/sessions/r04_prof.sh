#!/bin/bash
# round-4 evidence (profiles/r04/end/): FETCH/WRITE/L2 counter passes of the bench
# command for xsort (headline) and CSR5 (config3's kernel) -> profiles/pmc_{xsort,csr5}.json,
# the default bench line, and rocprofv3 kernel-trace stats of that same command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_prof
mkdir -p $O
T="timeout -k 10"
pmc() { # algo kernels alg_bytes extra-args
  local a=$1 k=$2 b=$3; shift 3
  local P="bench.py --no-cpu-baseline --no-rowsplit-beside --no-config3 --steps 5 --warmup 2 $*"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/$a/fetch -o run --output-format csv -- python3 $P > $O/$a.fetch.log 2>&1 || { tail -5 $O/$a.fetch.log; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/$a/write -o run --output-format csv -- python3 $P > $O/$a.write.log 2>&1 || { tail -5 $O/$a.write.log; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/$a/l2 -o run --output-format csv -- python3 $P > $O/$a.l2.log 2>&1 || { tail -5 $O/$a.l2.log; return 1; }
  python3 s-blas_amd/tools/pmc_traffic.py --kernel $k --fetch $O/$a/fetch --write $O/$a/write --l2 $O/$a/l2 --algorithmic $b --out $O/pmc_$a.json
}
pmc xsort k_spmv_xsort,k_xsort_reduce 533000004 && pmc csr5 k_spmv_csr5,k_csr5_calibrate 533000004 --algo csr5 || exit 1
cp $O/pmc_xsort.json profiles/pmc_xsort.json && cp $O/pmc_csr5.json profiles/pmc_csr5.json
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
$T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cat $O/pmc_xsort.json $O/pmc_csr5.json; head -c 600 $O/bench_default.json
