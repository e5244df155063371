#!/bin/bash
# round 5: pull SpTRSV grid size below one workgroup per CU (SBLAS_TRSV_GRID,
# experiment): level order at 64 threads on the stencils, natural order at
# 128 threads on the config-5 stand-in -> profiles/r05/trsv_waves/grid_*.json
set -o pipefail
O=gpurun_out/r05_trsv6
mkdir -p $O
T="timeout -k 10 150"
for M in "s27" "s7" "c5"; do
  case $M in c5) A="";; s27) A="--stencil 100 --points 27";; s7) A="--stencil 100 --points 7";; esac
  for g in 256 192 128 96 64 384; do
    SBLAS_TRSV_GRID=$g $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline $A > $O/grid_${M}_$g.json 2> $O/grid_${M}_$g.err || { tail -5 $O/grid_${M}_$g.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/grid_${M}_$g.json').read().strip().splitlines()[-1]); r=d['executors']
print('$M grid $g', {k: r[k]['ms'] for k in ('pull_csr', 'pull_level_order', 'pull_auto')})"
  done
done
