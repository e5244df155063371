# SpMM MFMA fill threshold default 0.15: every SpMM test; 7-point stencil at
# the default (row forms: its 16-row blocks fill ~8.5%) vs forced MFMA (0.08)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_spmm_fill
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "spmm or csrmm" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="s-blas_amd/tools/bench_spmm.py --stencil 150 --points 7 --no-cpu-baseline --steps 10"
for f in 0.15 0.08; do
  SBLAS_SPMM_MFMA_FILL=$f $T 400 python $B --check > $O/bench7_fill$f.json 2> $O/bench7_fill$f.err || { tail -20 $O/bench7_fill$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench7_fill$f.json')); print('7pt fill $f', d['kernel_ms_max_over_ranks'], d['value'], d['roofline']['frac'], d.get('check_vs_oracle', {}).get('pass'))"
done
$T 400 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > $O/bench_cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4', d['kernel_ms_max_over_ranks'], d['value'], d['roofline']['frac'])"
echo done
