# SpTRSV/SpTRSM poll back-off: tests at the new defaults, then SBLAS_TRSV_SLEEP
# 1 / -3 / -6 on the stencil triangles (level order) at rhs 1, 8, 64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_sleep
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "trsv or trsm or sptrsv or config5" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sl in default 1 -3 -6; do
for a in "--stencil 100 --points 27" "--stencil 100 --points 7" ""; do
  tag=s$sl$(echo "x$a" | tr -d ' -')
  if [ $sl = default ]; then E=""; else E="SBLAS_TRSV_SLEEP=$sl"; fi
  env $E $T 300 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 8,64 --no-push-rhs --steps 5 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', {k: v['ms'] for k, v in d['executors'].items() if 'auto' in k})"
done
done
echo done
