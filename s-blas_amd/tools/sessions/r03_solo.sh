# solo narrow items (SBLAS_XS_SOLO=1: a narrow range of up to 16,384 rows is
# an item of its own, wide ranges pair) vs the default pairing: parity, the
# default bench line, rank-0 slices
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_solo
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "solo" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="bench.py --no-cpu-baseline --no-rowsplit-beside"
for i in 1 2; do
  $T 300 python $B > $O/bench_base_$i.json 2> $O/bench_base_$i.err || { tail -20 $O/bench_base_$i.err; exit 1; }
  SBLAS_XS_SOLO=1 $T 300 python $B > $O/bench_solo_$i.json 2> $O/bench_solo_$i.err || { tail -20 $O/bench_solo_$i.err; exit 1; }
done
for f in $O/bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['kernel_ms'], d['roofline']['frac'], d['warm']['kernel_ms'])"; done
S="s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort"
run() { # name, env...
  local n=$1; shift
  env "$@" $T 300 python $S > $O/slice_$n.jsonl 2> $O/slice_$n.err || { tail -20 $O/slice_$n.err; exit 1; }
  echo "== $n"; cat $O/slice_$n.jsonl
}
run base SBLAS_XS_SOLO=0
run solo SBLAS_XS_SOLO=1
echo done
