# row split with lane-consecutive entries (SBLAS_RS_SEQ=1) vs 4 consecutive
# entries per lane: parity, then the row-split line on each matrix class
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_rsseq
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "rowsplit" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="bench.py --algo rowsplit --no-cpu-baseline --no-rowsplit-beside"
for m in "--matrix stencil7" "--matrix stencil27" "--matrix synth" "--matrix synth --cols prefix" "--matrix rmat"; do
  tag=$(echo $m | tr -d ' -' )
  for q in 0 1; do
    SBLAS_RS_SEQ=$q $T 400 python $B $m > $O/bench_${tag}_seq$q.json 2> $O/bench_${tag}_seq$q.err || { tail -20 $O/bench_${tag}_seq$q.err; exit 1; }
  done
done
for f in $O/bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['config']['algo'], d['kernel_ms'], d['roofline']['frac'])"; done
echo done
