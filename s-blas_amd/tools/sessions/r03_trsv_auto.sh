# SpTRSV algo 4 (AUTO ticket order): tests, then stencil triangles and the
# config-5 stand-in with every executor
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsv_auto
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "sptrsv or trsv or config5" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "--stencil 100 --points 27" "--stencil 100 --points 7" ""; do
  tag=$(echo "x$a" | tr -d ' -')
  $T 400 python s-blas_amd/tools/bench_sptrsv.py $a --steps 3 > $O/trsv_$tag.json 2> $O/trsv_$tag.err || { tail -20 $O/trsv_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsv_$tag.json'))
print('$tag', d['config']['n'], d['config']['levels'], d['config']['auto_pull_order'], {k: v['ms'] for k, v in d['executors'].items()}, d.get('cpu_baseline'))"
done
echo done
