#!/bin/bash
# round 5: C-tile SpMM with half-height tiles (SBLAS_SPMM_CTR=602: two
# workgroups' tiles fit a CU's LDS) and 1 or 2 slab sets, config 4 cold,
# alternating with the default -> profiles/r05/spmm_tiles/
set -o pipefail
O=gpurun_out/r05_spmm3
mkdir -p $O
T="timeout -k 10 200"
run() {
  local tag=$1; shift
  env "$@" $T python s-blas_amd/tools/bench_spmm_slices.py --worlds 1 --reps 8 > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  grep -h summary $O/$tag.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['kernel_max_us'])"
}
for r in 1 2; do
  run def$r SBLAS_SPMM_DUMMY=0 || exit 1
  run r602ns2_$r SBLAS_SPMM_CTR=602 SBLAS_SPMM_CTNS=2 || exit 1
  run r602ns1_$r SBLAS_SPMM_CTR=602 SBLAS_SPMM_CTNS=1 || exit 1
  run r602ns4_$r SBLAS_SPMM_CTR=602 SBLAS_SPMM_CTNS=4 || exit 1
done
