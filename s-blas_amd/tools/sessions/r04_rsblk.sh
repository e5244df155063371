#!/bin/bash
# round 4: row-split stream blocks of 4096 nnz (16 entries per thread; alt build) vs 2048
set -o pipefail
O=gpurun_out/r04_rsblk; mkdir -p $O
ALT=$PWD/s-blas_amd/alt/libsblas.so
SBLAS_LIB=$ALT timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_spmv_gpu.py -k "rowsplit or panel" \
  > $O/tests_alt.log 2>&1 || { echo ALT TESTS FAILED; tail -30 $O/tests_alt.log; exit 1; }
tail -1 $O/tests_alt.log
for i in 1 2; do
  timeout -k 10 300 python s-blas_amd/tools/exp_split.py --variants rowsplit,panel > $O/def_$i.jsonl 2>>$O/err.log || exit 1
  SBLAS_LIB=$ALT timeout -k 10 300 python s-blas_amd/tools/exp_split.py --variants rowsplit,panel > $O/alt_$i.jsonl 2>>$O/err.log || exit 1
  for f in def alt; do python3 -c "import json;print('$f', [(d['part'],d['variant'],d['cold_us']) for d in map(json.loads,open('$O/${f}_$i.jsonl'))])"; done
done
