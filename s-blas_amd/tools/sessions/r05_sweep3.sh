#!/bin/bash
# round 5: xsort at N = 1 on the uniform matrix, deeper claims and the
# layouts combined with U = 2, two alternations -> profiles/r05/sweep3/
set -o pipefail
O=gpurun_out/r05_sweep3
mkdir -p $O
run() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py "$@" --reps 6 > $O/$tag.jsonl 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; return 1; }
  python3 -c "
import json
for l in open('$O/$tag.jsonl'):
    d=json.loads(l); print('$tag', d['world'], d['algo'], d['cold_span_us'], d['warm_us'])"
}
X="--worlds 1 --algos xsort"
for i in 1 2; do
  run def$i -- $X && run u3_$i SBLAS_XS_U=3 -- $X && run u4_$i SBLAS_XS_U=4 -- $X && \
  run solo$i SBLAS_XS_SOLO=1 -- $X && run unp$i SBLAS_XS_PAIR=0 -- $X && run lam05_$i SBLAS_XS_LAMBDA=0.5 -- $X || exit 1
done
