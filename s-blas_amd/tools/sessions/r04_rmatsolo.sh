#!/bin/bash
# round 4: xsort takes solo narrow items on matrices with >= 40% empty rows (R-MAT):
# parity (spmv + SuiteSparse-class tests), R-MAT / config 2 / stencil spans
set -o pipefail
O=gpurun_out/r04_rmatsolo; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --tag auto$i >> $O/rmat.jsonl 2>>$O/err.log || exit 1
  SBLAS_XS_SOLO=0 timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --tag paired$i >> $O/rmat.jsonl 2>>$O/err.log || exit 1
done
python3 -c "
import json
for l in open('$O/rmat.jsonl'):
    d=json.loads(l); print(d['tag'], d['cold_span_us'], d['frac_8TBs'])"
B="--no-cpu-baseline --no-rowsplit-beside --no-config3"
for mtx in synth stencil27 stencil7 rmat; do
  timeout -k 10 300 python bench.py --matrix $mtx --check $B > $O/bench_$mtx.json 2>>$O/err.log || exit 1
  python3 -c "
import json; d=json.loads(open('$O/bench_$mtx.json').read().strip().splitlines()[-1]); print('$mtx', d['config']['algo'], d['ms_per_step'], d['roofline']['frac'], d.get('check'))"
done
