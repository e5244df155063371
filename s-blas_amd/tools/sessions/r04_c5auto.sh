#!/bin/bash
# round 4: CSR5 picks XCD column panels on scattered columns (probe shared with AUTO)
set -o pipefail
O=gpurun_out/r04_c5auto; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_spmv_gpu.py tests/test_configs_gpu.py \
  tests/test_bench_gpu.py tests/test_ctx_gpu.py -k "not trsv and not spmm and not transpose" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos csr5 > $O/slice_auto.jsonl 2>>$O/err.log || exit 1
SBLAS_CSR5_PANEL=0 timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos csr5 > $O/slice_plain.jsonl 2>>$O/err.log || exit 1
for f in auto plain; do python3 -c "import json;print('$f', [(d['world'],d['cold_span_us']) for d in map(json.loads,open('$O/slice_$f.jsonl'))])"; done
timeout -k 10 300 python bench.py > $O/bench_default.json 2>>$O/err.log || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['frac'], d['config3']['kernel_ms_max'], d['config3']['roofline']['frac'])"
for m in stencil27 stencil7; do
  timeout -k 10 300 python bench.py --matrix $m --algo csr5 --no-config3 --no-cpu-baseline --no-rowsplit-beside > $O/bench_$m.json 2>>$O/err.log || exit 1
  python3 -c "import json;d=json.loads(open('$O/bench_$m.json').read().strip().splitlines()[-1]);print('$m csr5', d['ms_per_step'], d['roofline']['frac'])"
done
