#!/bin/bash
# round 4: CSR5 tiles of 64 x sigma entries, sigma = 8 / 32 (alt builds) vs 16:
# parity on the alt builds, then config 2 (panels), configs[2]'s N = 8 heavy / light
# ranks, the stencils
set -o pipefail
O=gpurun_out/r04_c5sigma; mkdir -p $O
for v in s8 s32; do
  case $v in s8) L=$PWD/s-blas_amd/alt8/libsblas.so;; s32) L=$PWD/s-blas_amd/alt/libsblas.so;; esac
  SBLAS_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_spmv_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "csr5 or forms" > $O/tests_$v.log 2>&1 || { echo $v; tail -20 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
for i in 1 2; do
  for v in s16 s8 s32; do
    unset SBLAS_LIB
    case $v in s8) export SBLAS_LIB=$PWD/s-blas_amd/alt8/libsblas.so;; s32) export SBLAS_LIB=$PWD/s-blas_amd/alt/libsblas.so;; esac
    timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos csr5 --partition nnz --ranks 0,5 > $O/${v}_$i.jsonl 2>>$O/err.log || exit 1
    timeout -k 10 300 python bench.py --matrix stencil27 --algo csr5 --no-cpu-baseline --no-rowsplit-beside --no-config3 > $O/st27_${v}_$i.json 2>>$O/err.log || exit 1
    python3 -c "
import json
out=[(d['world'], d['rank'], d['cold_span_us']) for d in map(json.loads, open('$O/${v}_$i.jsonl'))]
d=json.loads(open('$O/st27_${v}_$i.json').read().strip().splitlines()[-1]); out.append(('st27', d['ms_per_step']))
print('$v$i', out)"
  done
done
