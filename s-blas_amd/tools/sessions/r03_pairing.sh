# leftover light sub-items paired only as far as the grid needs (planner):
# xsort parity, R-MAT / stencil / default lines, rank slices
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_pairing
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "xsort or suitesparse_class or config2" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in rmat stencil7; do
  $T 400 python bench.py --matrix $m --no-cpu-baseline --no-rowsplit-beside > $O/bench_${m}.json 2> $O/bench_${m}.err || { tail -20 $O/bench_${m}.err; exit 1; }
done
$T 400 python bench.py --matrix rmat --check --no-cpu-baseline --no-rowsplit-beside --steps 3 > $O/bench_rmat_check.json 2> $O/rmat_check.err || { tail -20 $O/rmat_check.err; exit 1; }
$T 400 python bench.py --no-cpu-baseline --no-rowsplit-beside > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
for f in $O/bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['config']['algo'], d['value'], d['kernel_ms'], d['roofline']['frac'], d.get('check_vs_oracle'))"; done
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort > $O/slice.jsonl 2> $O/slice.err || { tail -20 $O/slice.err; exit 1; }
cat $O/slice.jsonl
echo done
