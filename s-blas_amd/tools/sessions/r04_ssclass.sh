#!/bin/bash
# round 4: every SpMV kernel on the SuiteSparse-class generators (bench.py --matrix),
# cold spans with --check, the final tree
set -o pipefail
O=gpurun_out/r04_ssclass; mkdir -p $O
B="--no-cpu-baseline --no-rowsplit-beside --no-config3 --check"
for mtx in stencil27 stencil7 rmat; do
  for a in rowsplit csr5 panel xsort; do
    timeout -k 10 300 python bench.py --matrix $mtx --algo $a $B > $O/bench_${mtx}_$a.json 2>>$O/err.log || exit 1
    python3 -c "
import json; d=json.loads(open('$O/bench_${mtx}_$a.json').read().strip().splitlines()[-1]); print('$mtx $a', d['ms_per_step'], d['roofline']['frac'], d['check_vs_oracle'])"
  done
done
