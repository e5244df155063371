#!/bin/bash
# round 4: A/B of the bounded CSR5 staging run (default build) against HEAD's
# spmv.hip (alt build), alternated twice: config 2, slices, stencils
set -o pipefail
O=gpurun_out/r04_c5occ2; mkdir -p $O
for v in def1 alt1 def2 alt2; do
  unset SBLAS_LIB
  case $v in alt*) export SBLAS_LIB=$PWD/s-blas_amd/alt/libsblas.so;; esac
  timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos csr5 > $O/slice_$v.jsonl 2>>$O/err.log || exit 1
  timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 8 --algos csr5 --partition nnz --ranks 0,5 > $O/nnz_$v.jsonl 2>>$O/err.log || exit 1
  for mtx in stencil27 stencil7; do
    timeout -k 10 300 python bench.py --matrix $mtx --algo csr5 --no-cpu-baseline --no-rowsplit-beside --no-config3 > $O/bench_${mtx}_$v.json 2>>$O/err.log || exit 1
  done
  python3 -c "
import json
out=[(d['world'], d['rank'], d['cold_span_us']) for f in ('slice','nnz') for d in map(json.loads, open('$O/'+f+'_$v.jsonl'))]
for mtx in ('stencil27','stencil7'):
    d=json.loads(open('$O/bench_'+mtx+'_$v.json').read().strip().splitlines()[-1]); out.append((mtx, d['ms_per_step'], d['roofline']['frac']))
print('$v', out)"
done
