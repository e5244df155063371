# round 3: N = 8 slice, kernel-trace breakdown of the xsort variants (default, all-wide)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_slice
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort > $O/slice_default.jsonl 2> $O/e1.err &&
SBLAS_XS_ALLWIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_allwide -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort > $O/slice_allwide.jsonl 2> $O/e2.err
echo rc=$?
cat $O/slice_*.jsonl
for d in default allwide; do echo $d; python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$d/run_kernel_stats.csv')):
    if 'sblas' in r['Name']: print('  ', r['Name'][:60], r['Calls'], r['AverageNs'])
"; done
