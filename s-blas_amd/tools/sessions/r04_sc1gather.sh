#!/bin/bash
# round 4: xsort gathers as sc1 loads (L1 bypassed, L2-served; SBLAS_XS_MODE=32) vs plain
set -o pipefail
O=gpurun_out/r04_sc1gather; mkdir -p $O
SBLAS_XS_MODE=32 timeout -k 10 300 python -u -m pytest tests/test_spmv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "xsort and not k24 and not batch" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort > $O/def_$i.jsonl 2>>$O/err.log || exit 1
  SBLAS_XS_MODE=32 timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort > $O/sc1_$i.jsonl 2>>$O/err.log || exit 1
  for v in def sc1; do python3 -c "import json;print('$v$i', [(d['world'],d['cold_span_us']) for d in map(json.loads,open('$O/${v}_$i.jsonl'))])"; done
done
