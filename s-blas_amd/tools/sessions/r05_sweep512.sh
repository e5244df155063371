#!/bin/bash
# round 5: planner knobs re-swept on the paired 512-thread default (config 2
# N = 1 / 8 slices, 27-point stencil) -> profiles/r05/sweep512/
set -o pipefail
O=gpurun_out/r05_sweep512
mkdir -p $O
T="timeout -k 10 200"
run() {
  local tag=$1; shift
  env "$@" $T python s-blas_amd/tools/bench_slice.py --worlds 1,8 --ranks 0 --algos xsort --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  env "$@" $T python s-blas_amd/tools/spmv_one.py --matrix stencil27 --grid 128 --algo xsort --reps 8 --cold --scrub read >> $O/${tag}_struct.txt 2>&1 || { tail -5 $O/${tag}_struct.txt; exit 1; }
  python3 -c "
import json
print('$tag', [(json.loads(l)['world'], json.loads(l)['cold_span_us']) for l in open('$O/$tag.jsonl')], [l.split('mean')[1][:10] for l in open('$O/${tag}_struct.txt') if 'mean' in l])"
}
for r in 1 2; do
  run def$r SBLAS_XS_DUMMY=0 || exit 1
  run solo$r SBLAS_XS_SOLO=1 || exit 1
  run q1_$r SBLAS_XS_Q=1 || exit 1
  run q4_$r SBLAS_XS_Q=4 || exit 1
  run lam05_$r SBLAS_XS_LAMBDA=0.5 || exit 1
  run lam2_$r SBLAS_XS_LAMBDA=2 || exit 1
  run wb05_$r SBLAS_XS_WBUDGET=0.5 || exit 1
done
