# SpTRSM pull: right-hand sides per lane (V) x workgroups per CU, after the
# SpTRSM tests at the default V
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_v
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "trsv or trsm or sptrsv or config5" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for vw in 1:1 2:1 4:1 4:2 4:4; do
v=${vw%:*}; w=${vw#*:}
for a in "--stencil 100 --points 27" ""; do
  tag=v${v}w$w$(echo "x$a" | tr -d ' -')
  SBLAS_TRSM_V=$v SBLAS_TRSM_WG_PER_CU=$w $T 500 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 4,8,64 --no-push-rhs --steps 3 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', {k: (v['ms'], '%.0e' % v['rel_l1_vs_xref']) for k, v in d['executors'].items() if 'trsm' in k})"
done
done
echo done
