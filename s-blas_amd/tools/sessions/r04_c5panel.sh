#!/bin/bash
# round 4: staged CSR5 tile (gap tiles staged too) in the plain and the XCD-panel CSR5 forms
set -o pipefail
O=gpurun_out/r04_c5panel; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_spmv_gpu.py -k "csr5" \
  "tests/test_configs_gpu.py::test_config2_full_size" tests/test_kernels_gpu.py -k "csr5 or config2" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for F in 2 0; do
  SBLAS_C5_PF=$F timeout -k 10 300 python s-blas_amd/tools/exp_split.py --variants csr5,csr5p2,csr5p4,csr5p8 > $O/split_f$F.jsonl 2>>$O/err.log || exit 1
  python3 -c "import json;print('form $F', [(d['part'],d['variant'],d['cold_us']) for d in map(json.loads,open('$O/split_f$F.jsonl'))])"
done
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos csr5 > $O/slice.jsonl 2>>$O/err.log || exit 1
python3 -c "import json;print([(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/slice.jsonl'))])"
