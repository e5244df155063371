# SpMM MFMA tile, two chunks per step (loads of both issued first): SpMM tests,
# stencil lines with --check
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_spmm_unroll
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "spmm or csrmm" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pts in 27 7; do
  g=100; [ $pts = 7 ] && g=150
  $T 400 python s-blas_amd/tools/bench_spmm.py --stencil $g --points $pts --check --no-cpu-baseline --steps 10 > $O/bench_s$pts.json 2> $O/s$pts.err || { tail -20 $O/s$pts.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_s$pts.json')); print('$pts-pt', d['kernel_ms_max_over_ranks'], d['value'], d['roofline']['frac'], d['check_vs_oracle']['pass'])"
done
echo done
