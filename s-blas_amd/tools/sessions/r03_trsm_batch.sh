# SpTRSM pull with batched dependency loads (kBatch 8) and agent-scope polls on
# one device: tests, then the stencil triangles and the config-5 stand-in
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_batch
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "sptrsv or trsv or trsm or config5" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "--stencil 100 --points 27" "--stencil 100 --points 7" ""; do
  tag=$(echo "x$a" | tr -d ' -')
  $T 500 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 8,64 --no-push-rhs --steps 3 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', d['config']['n'], d['config']['auto_pull_order'], {k: v['ms'] for k, v in d['executors'].items()})"
done
echo done
