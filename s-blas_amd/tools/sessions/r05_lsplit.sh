#!/bin/bash
# round 5: split light ranges (SBLAS_XS_SOLO=1 SBLAS_XS_LSPLIT=S): xsort tests,
# then config 2 N = 1 and the N = 8 slice cold, alternating with the default
# -> profiles/r05/lsplit/
set -o pipefail
O=gpurun_out/r05_lsplit
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "xsort" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" SBLAS_XS_TIMING=1 $T 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --ranks 0 --algos xsort --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  grep "plan:.*ranges" $O/$tag.err | tail -2
  python3 -c "
import json
for l in open('$O/$tag.jsonl'):
    d=json.loads(l); print('$tag', d['world'], d['cold_span_us'])"
}
for r in 1 2; do
  run def$r SBLAS_XS_DUMMY=0 || exit 1
  run solo$r SBLAS_XS_SOLO=1 || exit 1
  run ls2_$r SBLAS_XS_SOLO=1 SBLAS_XS_LSPLIT=2 || exit 1
  run ls3_$r SBLAS_XS_SOLO=1 SBLAS_XS_LSPLIT=3 || exit 1
  run ls4_$r SBLAS_XS_SOLO=1 SBLAS_XS_LSPLIT=4 || exit 1
done
