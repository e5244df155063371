#!/bin/bash
# round 4: panel reduce with every partial load issued up front
set -o pipefail
O=gpurun_out/r04_pred; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_spmv_gpu.py tests/test_configs_gpu.py \
  -k "not trsv and not spmm and not transpose" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2 --algos rowsplit,csr5,panel > $O/slice.jsonl 2>>$O/err.log || exit 1
python3 -c "import json;print([(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/slice.jsonl'))])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/full -o run --output-format csv -- python3 s-blas_amd/tools/exp_split.py --parts full --variants csr5,rowsplit --reps 6 > $O/full.log 2>&1 || { tail -5 $O/full.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r04_pred/full/run_kernel_stats.csv')):
    n=r['Name']
    if any(k in n for k in ('csr5','panel','calibrate','rowsplit')): print(f"  {n[:50]:50s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:8.1f} us")
PY
