#!/bin/bash
# round 5: xsort with paired 512-thread workgroups (two 4-wave teams, up to
# 256 VGPRs; SBLAS_XS_WG=512p experiment) at 2 / 3 / 4 chunks per claim vs
# the default: xsort tests, config 2 N = 1 / 8 and the stencils, cold
# -> profiles/r05/wg512p/
set -o pipefail
O=gpurun_out/r05_wg512p
mkdir -p $O
T="timeout -k 10"
SBLAS_XS_WG=512p $T 600 python -u -m pytest tests/test_spmv_gpu.py -x -q --timeout 200 --timeout-method thread -k "xsort and not wg512 and not wg768 and not unpaired and not static" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" $T 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --ranks 0 --algos xsort --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  for M in "stencil27 --grid 128" "stencil7 --grid 160"; do
    env "$@" $T 200 python s-blas_amd/tools/spmv_one.py --matrix $M --algo xsort --reps 8 --cold --scrub read >> $O/${tag}_struct.txt 2>&1 || { tail -5 $O/${tag}_struct.txt; exit 1; }
  done
  python3 -c "
import json
print('$tag', [(json.loads(l)['world'], json.loads(l)['cold_span_us']) for l in open('$O/$tag.jsonl')], [l.split('mean')[1][:10] for l in open('$O/${tag}_struct.txt') if 'mean' in l])"
}
for r in 1 2; do
  run def$r SBLAS_XS_DUMMY=0 || exit 1
  run p512u2_$r SBLAS_XS_WG=512p SBLAS_XS_U=2 || exit 1
  run p512u3_$r SBLAS_XS_WG=512p SBLAS_XS_U=3 || exit 1
  run p512u4_$r SBLAS_XS_WG=512p SBLAS_XS_U=4 || exit 1
done
