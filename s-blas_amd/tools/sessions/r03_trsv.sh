# round 3: persistent multi-GPU SpTRSV handle -- parity, then config-5 bench with 4 blocks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsv
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "sptrsv or trsv or trsm" "tests/test_configs_gpu.py::test_config5_blocks_exact" "tests/test_configs_gpu.py::test_config5_real_vs_serial_oracle" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python s-blas_amd/tools/bench_sptrsv.py --mgpu 1,4 --no-cpu-baseline --steps 5 > $O/bench_sptrsv.json 2> $O/b.err
echo rc=$?
python3 -c "import json; d=json.loads(open('$O/bench_sptrsv.json').read().strip().splitlines()[-1]); print({k:v for k,v in d['executors'].items() if 'mgpu' in k})"
