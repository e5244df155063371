#!/bin/bash
# round 4: CSR5 staging run bounded to 512 slots (occupancy 4 -> 5 waves/SIMD) and an
# alt build asking for 6 (SBLAS_C5_WPE=6, small spills): parity, config 2, slices
# (cyclic rank 0 and configs[2]'s nnz ranks), stencils
set -o pipefail
O=gpurun_out/r04_c5occ; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "csr5 or c5 or CSR5 or slice" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in def alt; do
  if [ $v = alt ]; then export SBLAS_LIB=$PWD/s-blas_amd/alt/libsblas.so; fi
  timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos csr5 > $O/slice_$v.jsonl 2>>$O/err.log || exit 1
  timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 8 --algos csr5 --partition nnz --ranks 0,4,5 > $O/nnz_$v.jsonl 2>>$O/err.log || exit 1
  for mtx in stencil27 stencil7; do
    timeout -k 10 300 python bench.py --matrix $mtx --algo csr5 --no-cpu-baseline --no-rowsplit-beside --no-config3 > $O/bench_${mtx}_$v.json 2>>$O/err.log || exit 1
  done
  python3 -c "
import json
print('$v', [(d['world'], d['rank'], d['cold_span_us']) for f in ('slice','nnz') for d in map(json.loads, open('$O/'+f+'_$v.jsonl'))])
for mtx in ('stencil27','stencil7'):
    d=json.loads(open('$O/bench_'+mtx+'_$v.json').read().strip().splitlines()[-1]); print('$v', mtx, d['ms_per_step'], d['roofline']['frac'])"
done
