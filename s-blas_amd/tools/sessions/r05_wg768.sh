#!/bin/bash
# round 5: xsort with 768-thread workgroups (6 + 6 waves, 168 VGPRs a wave;
# SBLAS_XS_WG=768 experiment) at 2 / 3 chunks per claim: xsort tests, then
# config 2 (N = 1, N = 8 slice) and the 27-point stencil, cold, alternating
# with the default -> profiles/r05/wg768/
set -o pipefail
O=gpurun_out/r05_wg768
mkdir -p $O
T="timeout -k 10"
SBLAS_XS_WG=768 $T 600 python -u -m pytest tests/test_spmv_gpu.py -x -q --timeout 200 --timeout-method thread -k "xsort and not wg512 and not unpaired and not static" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" $T 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --ranks 0 --algos xsort --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  env "$@" $T 200 python s-blas_amd/tools/spmv_one.py --matrix stencil27 --algo xsort --reps 8 --cold --scrub read > $O/${tag}_s27.txt 2>&1 || { tail -5 $O/${tag}_s27.txt; exit 1; }
  python3 -c "
import json
print('$tag', [(json.loads(l)['world'], json.loads(l)['cold_span_us']) for l in open('$O/$tag.jsonl')], open('$O/${tag}_s27.txt').read().strip().splitlines()[-1][-60:])"
}
for r in 1 2; do
  run def$r SBLAS_XS_DUMMY=0 || exit 1
  run w768u2_$r SBLAS_XS_WG=768 SBLAS_XS_U=2 || exit 1
  run w768u3_$r SBLAS_XS_WG=768 SBLAS_XS_U=3 || exit 1
done
