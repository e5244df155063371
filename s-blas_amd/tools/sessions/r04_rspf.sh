#!/bin/bash
# round 4: row-split blocks with the first row's bounds / y prefetched (row split, panel, out-of-core share it)
set -o pipefail
O=gpurun_out/r04_rspf; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_spmv_gpu.py \
  "tests/test_configs_gpu.py::test_config2_full_size" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python s-blas_amd/tools/exp_split.py --variants rowsplit,panel,csr5 > $O/split_$i.jsonl 2>>$O/err.log || exit 1
  python3 -c "import json;print([(d['part'],d['variant'],d['cold_us']) for d in map(json.loads,open('$O/split_$i.jsonl'))])"
done
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 8 --algos rowsplit,panel,csr5 > $O/slice8.jsonl 2>>$O/err.log || exit 1
python3 -c "import json;print([(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/slice8.jsonl'))])"
