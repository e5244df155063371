#!/bin/bash
# round 4: the row split over XCD column panels on large scattered matrices
set -o pipefail
O=gpurun_out/r04_rspanel; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_spmv_gpu.py tests/test_configs_gpu.py \
  tests/test_kernels_gpu.py tests/test_ctx_gpu.py -k "not trsv and not spmm and not transpose and not trsm" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos rowsplit > $O/slice.jsonl 2>>$O/err.log || exit 1
python3 -c "import json;print([(d['world'],d['cold_span_us']) for d in map(json.loads,open('$O/slice.jsonl'))])"
timeout -k 10 300 python bench.py > $O/bench_default.json 2>>$O/err.log || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['frac'], d['rowsplit_beside'], d['config3']['kernel_ms_max'], d['config3']['roofline']['frac'])"
for m in stencil27 stencil7 rmat; do
  timeout -k 10 300 python bench.py --matrix $m --algo rowsplit --no-config3 --no-cpu-baseline --no-rowsplit-beside > $O/bench_$m.json 2>>$O/err.log || exit 1
  python3 -c "import json;d=json.loads(open('$O/bench_$m.json').read().strip().splitlines()[-1]);print('$m rowsplit', d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --cols prefix --algo rowsplit --no-config3 --no-cpu-baseline --no-rowsplit-beside > $O/bench_prefix.json 2>>$O/err.log || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_prefix.json').read().strip().splitlines()[-1]);print('prefix rowsplit', d['ms_per_step'], d['roofline']['frac'])"
