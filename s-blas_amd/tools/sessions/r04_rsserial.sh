#!/bin/bash
# round 4: row blocks bounded to 32 serial adds per row (power-law rows): parity,
# then the row split / panel on R-MAT, config 2 and the stencils
set -o pipefail
O=gpurun_out/r04_rsserial; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "rowsplit or panel or suitesparse or ooc or out_of_core" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--no-cpu-baseline --no-rowsplit-beside --no-config3 --check"
for mtx in rmat synth stencil27 stencil7; do
  for a in rowsplit panel; do
    timeout -k 10 300 python bench.py --matrix $mtx --algo $a $B > $O/bench_${mtx}_$a.json 2>>$O/err.log || exit 1
    python3 -c "
import json; d=json.loads(open('$O/bench_${mtx}_$a.json').read().strip().splitlines()[-1]); print('$mtx $a', d['ms_per_step'], d['roofline']['frac'], d['check_vs_oracle'])"
  done
done
