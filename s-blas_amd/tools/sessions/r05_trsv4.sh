#!/bin/bash
# round 5: poll back-off at the new wave counts (SBLAS_TRSV_SLEEP; natural
# order default 1, level order -6) -> profiles/r05/trsv_waves/sleep_*.json
set -o pipefail
O=gpurun_out/r05_trsv4
mkdir -p $O
T="timeout -k 10 150"
for M in "c5" "s27"; do
  case $M in c5) A="";; s27) A="--stencil 100 --points 27";; esac
  for sl in 1 0 2 4 -2 -4 -6 -8; do
    SBLAS_TRSV_SLEEP=$sl $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline $A > $O/sleep_${M}_$sl.json 2> $O/sleep_${M}_$sl.err || { tail -5 $O/sleep_${M}_$sl.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/sleep_${M}_$sl.json').read().strip().splitlines()[-1]); r=d['executors']
print('$M sleep $sl', {k: v['ms'] for k, v in r.items() if k.startswith('pull')})"
  done
done
