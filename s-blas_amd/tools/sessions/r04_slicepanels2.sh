#!/bin/bash
# round 4: per-kernel panel thresholds (row split from 4M entries, CSR5 from 8M): the
# slice choice tests, the config / spmv parity files, and the N = 2/4/8 slices again
set -o pipefail
O=gpurun_out/r04_slicepanels2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_spmv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 2,4,8 --algos csr5,rowsplit > $O/slice.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
python3 -c "import json;print([(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/slice.jsonl'))])"
