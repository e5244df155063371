# last-arriver wide reduce (SBLAS_XS_TAIL=1) vs the separate reduce launch:
# parity of the tail cases, then the default bench line and rank-0 slices
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_tail
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "tail" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="bench.py --no-cpu-baseline --no-rowsplit-beside"
for i in 1 2; do
  $T 300 python $B > $O/bench_base_$i.json 2> $O/bench_base_$i.err || { tail -20 $O/bench_base_$i.err; exit 1; }
  SBLAS_XS_TAIL=1 $T 300 python $B > $O/bench_tail_$i.json 2> $O/bench_tail_$i.err || { tail -20 $O/bench_tail_$i.err; exit 1; }
done
for f in $O/bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['kernel_ms'], d['roofline']['frac'], d['warm']['kernel_ms'])"; done
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort > $O/slice_base.jsonl 2> $O/slice_base.err || { tail -20 $O/slice_base.err; exit 1; }
SBLAS_XS_TAIL=1 $T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort > $O/slice_tail.jsonl 2> $O/slice_tail.err || { tail -20 $O/slice_tail.err; exit 1; }
cat $O/slice_base.jsonl $O/slice_tail.jsonl
echo done
