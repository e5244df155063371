#!/bin/bash
# round 5: narrow epilogue y loads issued before the barrier (4-wave teams)
# against the previous build (SBLAS_LIB=libsblas_a.so): xsort tests, config 2
# N = 1 / 2 / 4 / 8 slices, the structured stand-ins -> profiles/r05/earlyy/
set -o pipefail
O=gpurun_out/r05_earlyy
mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "xsort" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" $T python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --ranks 0 --algos xsort --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  for M in "stencil27 --grid 128" "stencil7 --grid 160" "rmat --scale 21"; do
    env "$@" $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo xsort --reps 8 --cold --scrub read >> $O/${tag}_struct.txt 2>&1 || { tail -5 $O/${tag}_struct.txt; exit 1; }
  done
  python3 -c "
import json
print('$tag', [(json.loads(l)['world'], json.loads(l)['cold_span_us']) for l in open('$O/$tag.jsonl')], [l.split('mean')[1][:10] for l in open('$O/${tag}_struct.txt') if 'mean' in l])"
}
for r in 1 2; do
  run base$r SBLAS_LIB=s-blas_amd/libsblas_a.so || exit 1
  run early$r SBLAS_XS_DUMMY=0 || exit 1
done
