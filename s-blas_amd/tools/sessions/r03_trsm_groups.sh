# SpTRSM grouped ticket claims (SBLAS_TRSM_GROUPS x SBLAS_TRSM_SLICES):
# tests, then config 5 and the 27-point stencil at rhs 8..64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_groups
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "sptrsm_cols_per_lane or sptrsm_kat or sptrsv_auto_order" \
    tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for gs in 0:16 8:4 8:16 8:64; do
g=${gs%:*}; sl=${gs#*:}
for a in "--stencil 100 --points 27" ""; do
  tag=g${g}s$sl$(echo "x$a" | tr -d ' -')
  if [ $g = 0 ]; then E=""; else E="SBLAS_TRSM_GROUPS=$g SBLAS_TRSM_SLICES=$sl"; fi
  env $E $T 300 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 8,16,32,64 --no-push-rhs --steps 5 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', {k.replace('trsm_pull_',''): v['ms'] for k, v in d['executors'].items() if 'auto_rhs' in k})"
done
done
echo done
