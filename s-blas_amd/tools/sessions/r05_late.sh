#!/bin/bash
# round 5: xsort with values issued beside their gathers (SBLAS_XS_MODE=32,
# experiment) at 2 / 3 chunks per claim: correctness on the xsort tests, then
# config 2 cold, alternating with the default -> profiles/r05/late/
set -o pipefail
O=gpurun_out/r05_late
mkdir -p $O
T="timeout -k 10"
SBLAS_XS_MODE=32 SBLAS_XS_U=3 $T 600 python -u -m pytest tests/test_spmv_gpu.py -x -q --timeout 200 --timeout-method thread -k "xsort and not wg512 and not static and not unpaired" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" $T 200 python s-blas_amd/tools/bench_slice.py --worlds 1 --ranks 0 --algos xsort --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
for l in open('$O/$tag.jsonl'):
    d=json.loads(l); print('$tag', d['world'], d['cold_span_us'])"
}
for r in 1 2; do
  run def$r SBLAS_XS_DUMMY=0 || exit 1
  run late2_$r SBLAS_XS_MODE=32 SBLAS_XS_U=2 || exit 1
  run late3_$r SBLAS_XS_MODE=32 SBLAS_XS_U=3 || exit 1
  run late4_$r SBLAS_XS_MODE=32 SBLAS_XS_U=4 || exit 1
done
