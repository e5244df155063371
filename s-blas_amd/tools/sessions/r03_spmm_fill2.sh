# SpMM MFMA fill threshold default 0.08: every SpMM / csrmm test, the stencil
# lines at the default, config 4 unchanged (rail-like blocks fill ~1/16)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_spmm_fill2
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "spmm or csrmm" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pts in 27 7; do
  $T 400 python s-blas_amd/tools/bench_spmm.py --stencil 120 --points $pts --check --no-cpu-baseline --steps 10 > $O/bench_stencil$pts.json 2> $O/s$pts.err || { tail -20 $O/s$pts.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_stencil$pts.json')); print('$pts-pt', d['kernel_ms_max_over_ranks'], d['value'], d['roofline']['frac'], d['check_vs_oracle']['pass'])"
done
$T 400 python s-blas_amd/tools/bench_spmm.py > $O/bench_cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4', d['kernel_ms_max_over_ranks'], d['value'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
echo done
