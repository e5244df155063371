# round 3: SBLAS_SPMV_AUTO (sblas_csr_pick) -- parity tests and the bench lines it picks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_auto
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py tests/test_ctx_gpu.py tests/test_bench_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "auto or qh768 or synthetic or ctx or bench or config2" > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_auto_random.json 2> $O/e1.err &&
timeout -k 10 300 python bench.py --cols prefix --no-cpu-baseline > $O/bench_auto_prefix.json 2> $O/e2.err
rc=$?
tail -3 $O/tests.log
python3 -c "
import json
for f in ('random','prefix'):
    try:
        d=json.load(open('$O/bench_auto_%s.json'%f)); print(f, d['config']['algo'], d['value'], d['roofline']['frac'])
    except Exception as e: print(f, 'missing', e)
"
echo rc=$rc
