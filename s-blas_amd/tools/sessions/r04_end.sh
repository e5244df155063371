#!/bin/bash
# round-4 end evidence (profiles/r04/end/): FETCH/WRITE/L2 passes of the bench command for
# xsort (headline) and CSR5 (config3's kernel, XCD panels) -> profiles/pmc_{xsort,csr5}.json,
# the default bench line, and rocprofv3 kernel-trace stats of that same command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_end
mkdir -p $O
T="timeout -k 10"
pmc() { # name kernels alg_bytes extra-args
  local a=$1 k=$2 b=$3; shift 3
  local P="bench.py --no-cpu-baseline --no-rowsplit-beside --no-config3 --steps 5 --warmup 2 $*"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/$a/fetch -o run --output-format csv -- python3 $P > $O/$a.fetch.log 2>&1 || { tail -5 $O/$a.fetch.log; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/$a/write -o run --output-format csv -- python3 $P > $O/$a.write.log 2>&1 || { tail -5 $O/$a.write.log; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/$a/l2 -o run --output-format csv -- python3 $P > $O/$a.l2.log 2>&1 || { tail -5 $O/$a.l2.log; return 1; }
  python3 s-blas_amd/tools/pmc_traffic.py --kernel $k --fetch $O/$a/fetch --write $O/$a/write --l2 $O/$a/l2 --algorithmic $b --out $O/pmc_$a.json
}
pmc xsort k_spmv_xsort,k_xsort_reduce 533000004 && \
  pmc csr5 "k_spmv_csr5_panel<2>,k_csr5_calibrate_panel,k_panel_reduce<true>" 533000004 --algo csr5 && \
  pmc rowsplit "k_spmv_panel<false>,k_panel_reduce<true>" 533000004 --algo rowsplit || exit 1
cp $O/pmc_xsort.json profiles/pmc_xsort.json && cp $O/pmc_csr5.json profiles/pmc_csr5.json && cp $O/pmc_rowsplit.json profiles/pmc_rowsplit.json
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
$T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
$T 300 python bench.py --driver ctx > $O/bench_ctx1.json 2> $O/bench_ctx1.err || { tail -20 $O/bench_ctx1.err; exit 1; }
for a in xsort csr5 rowsplit; do python3 -c "import json;d=json.load(open('$O/pmc_$a.json'));print('$a', d['traffic_over_algorithmic'], d['l2_hit_rate'])"; done
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'], d['rowsplit_beside'], d['config3']['roofline'], d['cpu_baseline']['value'])"
