# SuiteSparse-class matrices (bench.py --matrix): 3-D 7/27-point stencils and an
# R-MAT power-law graph, every kernel's parity, then the bench line per kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_ssclass
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "suitesparse_class or auto_pick" \
    tests/test_spmv_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in stencil7 stencil27 rmat; do
  $T 400 python bench.py --matrix $m --no-rowsplit-beside > $O/bench_${m}_auto.json 2> $O/bench_${m}_auto.err || { tail -20 $O/bench_${m}_auto.err; exit 1; }
  for a in rowsplit csr5 xsort panel; do
    $T 400 python bench.py --matrix $m --algo $a --no-cpu-baseline --no-rowsplit-beside > $O/bench_${m}_$a.json 2> $O/bench_${m}_$a.err || { tail -20 $O/bench_${m}_$a.err; exit 1; }
  done
done
for f in $O/bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['config']['algo'], d['value'], d['kernel_ms'], d['roofline']['frac'], d.get('cpu_baseline', {}).get('value'))"; done
echo done
