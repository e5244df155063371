# lane-consecutive stream blocks as the default of every row-split user
# (row split, XCD panels, out-of-core chunks): parity, panel lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_rsseq2
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "rowsplit or panel or ooc or out_of_core or reference_api" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="bench.py --algo panel --no-cpu-baseline --no-rowsplit-beside"
for m in "--matrix stencil7" "--matrix stencil27" "--matrix synth"; do
  tag=$(echo $m | tr -d ' -' )
  $T 400 python $B $m > $O/bench_panel_${tag}.json 2> $O/bench_panel_${tag}.err || { tail -20 $O/bench_panel_${tag}.err; exit 1; }
done
$T 400 python bench.py --algo rowsplit --cols prefix --no-cpu-baseline --no-rowsplit-beside > $O/bench_rowsplit_prefix.json 2> $O/rp.err || { tail -20 $O/rp.err; exit 1; }
for f in $O/bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['config']['algo'], d['kernel_ms'], d['roofline']['frac'])"; done
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 8,16 --algos panel,rowsplit > $O/slice.jsonl 2> $O/slice.err || { tail -20 $O/slice.err; exit 1; }
cat $O/slice.jsonl
echo done
