#!/bin/bash
# round 4: CSR5 calibrate with its loads issued together: kernel stats on the N = 8
# heavy / light ranks and config 2, plus the CSR5 parity files
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_cal2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "csr5 or forms" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 0 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r$r -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos csr5 --partition nnz --ranks $r > $O/slice_r$r.jsonl 2>>$O/err.log || exit 1
  python3 -c "
import csv, json
d=json.loads(open('$O/slice_r$r.jsonl').read().strip().splitlines()[-1]); print('r$r span', d['cold_span_us'])
for row in csv.DictReader(open('$O/prof_r$r/run_kernel_stats.csv')):
    if 'calibrate' in row['Name'] or 'k_spmv_csr5' in row['Name'] or 'reduce' in row['Name']: print('r$r', row['Name'].split('(')[0][-45:], row['Calls'], row['AverageNs'])"
done
