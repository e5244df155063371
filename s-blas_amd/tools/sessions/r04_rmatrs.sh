#!/bin/bash
# round 4: where the row split's time goes on R-MAT (rocprofv3 kernel stats)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_rmatrs; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 s-blas_amd/tools/exp_rmat.py --algos rowsplit,csr5 > $O/rmat.jsonl 2>>$O/err.log || exit 1
cat $O/rmat.jsonl
python3 -c "
import csv
for row in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'sblas' in row['Name']: print(row['Name'].split('(')[0][-45:], row['Calls'], row['AverageNs'])"
