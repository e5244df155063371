# AUTO with the column-spread probe: pick tests, SuiteSparse-class parity, the
# bench line (auto) per matrix class, and the default config-2 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_ssclass2
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    -k "suitesparse_class or auto_pick or config2_auto or ctx_spmv_chain or ctx_config2_full_size" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py tests/test_ctx_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in stencil7 stencil27 rmat; do
  $T 400 python bench.py --matrix $m > $O/bench_${m}_auto.json 2> $O/bench_${m}_auto.err || { tail -20 $O/bench_${m}_auto.err; exit 1; }
done
$T 400 python bench.py --matrix stencil27 --algo xsort --check --no-cpu-baseline --no-rowsplit-beside --steps 5 > $O/bench_stencil27_xsort_check.json 2> $O/check.err || { tail -20 $O/check.err; exit 1; }
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
for f in $O/bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['config']['algo'], d['value'], d['kernel_ms'], d['roofline']['frac'], d.get('rowsplit_beside', {}).get('roofline_frac'), d.get('cpu_baseline', {}).get('value'), d.get('check_vs_oracle'))"; done
echo done
