# small dynamic tail items (SBLAS_XS_TAILFRAC permille of the entries):
# parity, the default line and rank-0 slices at 0 / 30 / 60 / 100 permille
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_tailfrac
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "tailfrac" \
    tests/test_spmv_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 0 30 60 100 0 30 60 100; do
  SBLAS_XS_TAILFRAC=$f $T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,4,8 --algos xsort > $O/slice_$f.jsonl 2> $O/slice_$f.err || { tail -20 $O/slice_$f.err; exit 1; }
  echo "== $f"; cat $O/slice_$f.jsonl
done
echo done
