#!/bin/bash
# round 5: paired 512-thread xsort (SBLAS_XS_WG=512p, planner's U) vs the
# default over config 2's N = 1 / 2 / 4 / 8 slices and the three structured
# stand-ins, cold, alternating -> profiles/r05/wg512p/
set -o pipefail
O=gpurun_out/r05_wg512pb
mkdir -p $O
T="timeout -k 10 200"
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
  run def$r SBLAS_XS_DUMMY=0 || exit 1
  run p512_$r SBLAS_XS_WG=512p || exit 1
done
