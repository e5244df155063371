#!/bin/bash
# round 5: xsort with 19,456 LDS row accumulators (`make alt`) vs 16,384 on
# the uniform config 2 (N = 1 and the N = 8 slice), alternating
# -> profiles/r05/lds19k/
set -o pipefail
O=gpurun_out/r05_lds19k; mkdir -p $O
ALT=$PWD/s-blas_amd/alt/libsblas.so
T="timeout -k 10"
SBLAS_LIB=$ALT $T 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_spmv_gpu.py -k "xsort" > $O/tests_alt.log 2>&1 || { tail -30 $O/tests_alt.log; exit 1; }
tail -1 $O/tests_alt.log
for i in 1 2; do
  $T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --ranks 0 --algos xsort --reps 8 > $O/def_$i.jsonl 2>>$O/err.log || exit 1
  SBLAS_LIB=$ALT $T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --ranks 0 --algos xsort --reps 8 > $O/alt_$i.jsonl 2>>$O/err.log || exit 1
  for f in def_$i alt_$i; do python3 -c "
import json
print('$f', [(json.loads(l)['world'], json.loads(l)['cold_span_us']) for l in open('$O/$f.jsonl')])"; done
done
