#!/bin/bash
# round 4: kernel breakdown of CSR5 on configs[2]'s N = 8 light rank (2 panels) and a
# heavy rank (plain): rocprofv3 kernel stats of bench_slice on each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_lightprof; mkdir -p $O
for r in 5 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r$r -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos csr5 --partition nnz --ranks $r > $O/slice_r$r.jsonl 2>>$O/err.log || exit 1
  python3 -c "
import csv
for row in csv.DictReader(open('$O/prof_r$r/run_kernel_stats.csv')):
    if 'sblas' in row['Name']: print('r$r', row['Name'].split('(')[0][-45:], row['Calls'], row['AverageNs'])"
done
