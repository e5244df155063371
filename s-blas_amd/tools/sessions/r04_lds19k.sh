#!/bin/bash
# round 4: xsort with 19,456 LDS row accumulators (160 KiB CU) vs 16,384 (default)
set -o pipefail
O=gpurun_out/r04_lds19k; mkdir -p $O
ALT=$PWD/s-blas_amd/alt/libsblas.so
SBLAS_LIB=$ALT timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_spmv_gpu.py -k "xsort" "tests/test_configs_gpu.py::test_config2_full_size" \
  "tests/test_configs_gpu.py::test_config2_rank_slice_xsort" > $O/tests_alt.log 2>&1 || { echo ALT TESTS FAILED; tail -40 $O/tests_alt.log; exit 1; }
tail -2 $O/tests_alt.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-config3 --no-cpu-baseline --no-rowsplit-beside > $O/bench_def_$i.json 2>>$O/err.log || exit 1
  SBLAS_LIB=$ALT timeout -k 10 200 python bench.py --no-config3 --no-cpu-baseline --no-rowsplit-beside > $O/bench_alt_$i.json 2>>$O/err.log || exit 1
done
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort > $O/slice_def.jsonl 2>>$O/err.log || exit 1
SBLAS_LIB=$ALT timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort > $O/slice_alt.jsonl 2>>$O/err.log || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r04_lds19k/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'], d['roofline']['frac'])
for f in ('slice_def','slice_alt'):
    for l in open(f'gpurun_out/r04_lds19k/{f}.jsonl'):
        d=json.loads(l); print(f, {k:d[k] for k in d if k in ('world','algo','cold_ms','warm_ms','cold_us','warm_us')} or l[:200])
PY
