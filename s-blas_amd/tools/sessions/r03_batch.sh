# round 3: batch form of the column-sorted kernel for small items (rank slices)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_batch
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_spmv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "xsort or slice" > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort > $O/slice_batch.jsonl 2> $O/e1.err &&
SBLAS_XS_BATCH=0 timeout -k 10 300 python3 s-blas_amd/tools/bench_slice.py --worlds 4,8 --algos xsort > $O/slice_persistent.jsonl 2> $O/e2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_batch -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort > $O/slice_prof.jsonl 2> $O/e3.err
rc=$?
tail -3 $O/tests.log
cat $O/slice_*.jsonl
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_batch/run_kernel_stats.csv')):
    if 'sblas' in r['Name']: print('  ', r['Name'][:60], r['Calls'], r['AverageNs'])
" 2>/dev/null
echo rc=$rc
