# SpTRSM pull at the default V choice: SpTRSM/SpTRSV tests, then stencil
# triangles and the config-5 stand-in at rhs 4..64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_vdef3
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "trsv or trsm or sptrsv or config5" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "--stencil 100 --points 27" "--stencil 100 --points 7" ""; do
  tag=$(echo "x$a" | tr -d ' -')
  $T 500 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 4,8,16,32,64 --steps 3 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', d['config']['auto_pull_order'], {k.replace('trsm_',''): v['ms'] for k, v in d['executors'].items() if 'trsm' in k})"
done
echo done
