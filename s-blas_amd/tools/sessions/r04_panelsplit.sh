#!/bin/bash
# round 4: wave-per-row panel split for rows >= 256 entries: parity, then the split's
# kernel times on R-MAT (rocprofv3) and the SpMV spans (unchanged expected)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_panelsplit; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "panel or csr5 or rowsplit or suitesparse" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 s-blas_amd/tools/exp_rmat.py --algos rowsplit,csr5 > $O/rmat.jsonl 2>>$O/err.log || exit 1
cat $O/rmat.jsonl
python3 -c "
import csv
for row in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'panel_' in row['Name']: print(row['Name'].split('(')[0][-45:], row['Calls'], row['AverageNs'])"
