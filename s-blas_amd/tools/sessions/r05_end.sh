#!/bin/bash
# round-5 end evidence (profiles/r05/end/): FETCH / WRITE / L2 passes of the
# default bench command -> profiles/pmc_{xsort,csr5,rowsplit,spmm_ctile}.json
# (stamped with the libsblas.so sha256 they ran), then the default bench line
# (whose roofline.traffic those stamps now validate), rocprofv3 kernel-trace
# stats of that same command (headline_kernels.json: the headline's own xsort
# launches; the stats csv also averages in the structured leg's), and the ctx
# driver's N = 1 line.  gpurun returns only gpurun_out/: copy
# gpurun_out/r05_end/pmc_*.json to profiles/ afterwards (the stamped summaries
# bench.py reads).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_end
mkdir -p $O
T="timeout -k 10"
P="bench.py --no-cpu-baseline --no-peak --steps 5 --warmup 2"
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d $O/pmc_$tag -o run --output-format csv -- python3 $P > $O/pmc_$tag.log 2>&1 || { tail -5 $O/pmc_$tag.log; exit 1; }
done
tr() { python3 s-blas_amd/tools/pmc_traffic.py --kernel "$2" --fetch $O/pmc_FETCH_SIZE --write $O/pmc_WRITE_SIZE --l2 $O/pmc_TCC_HIT_sum --algorithmic $3 --out $O/pmc_$1.json > /dev/null; }
tr xsort "k_spmv_xsort,k_xsort_reduce" 533000004 && \
  tr csr5 "k_spmv_csr5_panel<2>,k_csr5_calibrate_panel,k_panel_reduce<true>" 533000004 && \
  tr rowsplit "k_spmv_panel<false>,k_panel_reduce<true>" 533000004 && \
  tr spmm_ctile "k_spmm_ctile,k_spmm_ctreduce<true>" 699177252 || exit 1
for a in xsort csr5 rowsplit spmm_ctile; do cp $O/pmc_$a.json profiles/pmc_$a.json; done
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
$T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
$T 300 python bench.py --driver ctx --no-cpu-baseline > $O/bench_ctx1.json 2> $O/bench_ctx1.err || { tail -20 $O/bench_ctx1.err; exit 1; }
python3 s-blas_amd/tools/headline_kernels.py $O/prof/run_kernel_trace.csv --out $O/headline_kernels.json > /dev/null || exit 1
for a in xsort csr5 rowsplit spmm_ctile; do python3 -c "import json;d=json.load(open('$O/pmc_$a.json'));print('$a', round(d['traffic_over_algorithmic'],3), round(d['l2_hit_rate'],3))"; done
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'], d['traffic_source'], d['config3']['kernel_ms_max'], d['config4']['kernel_ms_max'], d['config5']['ms'], d['cpu_baseline']['value'])"
