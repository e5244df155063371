# SpTRSM pull, lane columns RP apart (coalesced): tests, then V in {1,2,4,8} at rhs 4..64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_v3
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "trsv or trsm or sptrsv or config5" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 2 4 8; do
for a in "--stencil 100 --points 27" ""; do
  tag=v${v}$(echo "x$a" | tr -d ' -')
  SBLAS_TRSM_V=$v $T 500 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 4,8,16,32,64 --no-push-rhs --steps 3 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', {k.replace('trsm_pull_',''): v['ms'] for k, v in d['executors'].items() if 'trsm' in k and 'auto' not in k})"
done
done
echo done
