#!/bin/bash
# round 5: pull SpTRSV waves per CU (SBLAS_TRSV_THREADS 64..256, one
# workgroup per CU) on the config-5 stand-in and two stencil triangles
# (level order) -> profiles/r05/trsv_waves/
set -o pipefail
O=gpurun_out/r05_trsv2
mkdir -p $O
T="timeout -k 10 150"
for M in "c5" "s27" "s7"; do
  case $M in c5) A="";; s27) A="--stencil 100 --points 27";; s7) A="--stencil 100 --points 7";; esac
  for t in 128 192 256 64 128; do
    SBLAS_TRSV_THREADS=$t $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline $A > $O/${M}_t$t.json 2> $O/${M}_t$t.err || { tail -5 $O/${M}_t$t.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${M}_t$t.json').read().strip().splitlines()[-1]); r=d['executors']
print('$M threads $t', {k: (v['ms'], v['rel_l1_vs_xref']) for k, v in r.items() if k.startswith('pull')})"
  done
done
