#!/bin/bash
# round 4: long-row chunks of 2048 entries (alt build) vs 8192 on R-MAT's row split
set -o pipefail
O=gpurun_out/r04_longchunk; mkdir -p $O
ALT=$PWD/s-blas_amd/alt/libsblas.so
SBLAS_LIB=$ALT timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "rowsplit or panel" > $O/tests_alt.log 2>&1 || { tail -20 $O/tests_alt.log; exit 1; }
tail -1 $O/tests_alt.log
for i in 1 2; do
  timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --algos rowsplit,panel --tag def$i >> $O/rmat.jsonl 2>>$O/err.log || exit 1
  SBLAS_LIB=$ALT timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --algos rowsplit,panel --tag alt$i >> $O/rmat.jsonl 2>>$O/err.log || exit 1
done
python3 -c "
import json
for l in open('$O/rmat.jsonl'):
    d=json.loads(l); print(d['tag'], d['algo'], d['cold_span_us'], d['frac_8TBs'])"
