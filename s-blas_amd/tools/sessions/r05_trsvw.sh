#!/bin/bash
# round 5: windowed pull SpTRSV (SBLAS_TRSV_FORM=1, one round trip per poll
# iteration) against k_trsv_pull: the SpTRSV tests under the form, then the
# config-5 stand-in and two stencil triangles, alternating -> profiles/r05/trsvw/
set -o pipefail
O=gpurun_out/r05_trsvw
mkdir -p $O
T="timeout -k 10 150"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "pull_form" > $O/tests_form.log 2>&1 || { tail -30 $O/tests_form.log; exit 1; }
tail -1 $O/tests_form.log
SBLAS_TRSV_FORM=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -k "trsv or sptrsv or config5" > $O/tests_all.log 2>&1 || { tail -30 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
for r in 1 2; do
for M in "c5" "s27" "s7"; do
  case $M in c5) A="";; s27) A="--stencil 100 --points 27";; s7) A="--stencil 100 --points 7";; esac
  for f in 0 1; do
    SBLAS_TRSV_FORM=$f $T python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline $A > $O/${M}_f${f}_$r.json 2> $O/${M}_f${f}_$r.err || { tail -5 $O/${M}_f${f}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${M}_f${f}_$r.json').read().strip().splitlines()[-1]); r=d['executors']
print('$M form $f', {k: (v['ms'], v['rel_l1_vs_xref']) for k, v in r.items() if k.startswith('pull')})"
  done
done
done
