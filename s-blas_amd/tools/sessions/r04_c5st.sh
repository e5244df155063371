#!/bin/bash
# round 4: CSR5 tile forms: 0 plain, 1 phased + prefetched row ends, 2 staged y (default)
set -o pipefail
O=gpurun_out/r04_c5st; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_spmv_gpu.py -k "csr5" \
  "tests/test_configs_gpu.py::test_config2_full_size" tests/test_kernels_gpu.py -k "csr5 or config2" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for F in 3 2 3 2; do
  SBLAS_C5_PF=$F timeout -k 10 300 python s-blas_amd/tools/exp_split.py --variants csr5 > $O/split_f$F.jsonl 2>>$O/err.log || exit 1
  python3 -c "import json;print('form $F', [(d['part'],d['cold_us']) for d in map(json.loads,open('$O/split_f$F.jsonl'))])"
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2>>$O/err.log || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['frac'], d['config3']['kernel_ms_max'], d['config3']['roofline']['frac'], d['cpu_baseline']['value'])"
