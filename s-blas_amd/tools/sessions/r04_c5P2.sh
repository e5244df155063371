#!/bin/bash
# round 4: CSR5 panel count by row length (2 panels from 4M entries on short rows,
# 4 from 8M otherwise): parity files, then configs[2]'s nnz-split ranks and config 2
set -o pipefail
O=gpurun_out/r04_c5P2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_spmv_gpu.py tests/test_bench_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos csr5 --partition nnz --ranks all > $O/auto.jsonl 2>>$O/err.log || exit 1
python3 -c "import json;print([(d['world'],d['rank'],d['cold_span_us']) for d in map(json.loads,open('$O/auto.jsonl'))])"
timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --algos csr5 --tag auto > $O/rmat.jsonl 2>>$O/err.log && cat $O/rmat.jsonl
