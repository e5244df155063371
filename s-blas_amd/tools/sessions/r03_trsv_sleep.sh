# SpTRSV pull poll back-off (SBLAS_TRSV_SLEEP) on the level-ordered stencil
# triangles and the config-5 stand-in
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsv_sleep${SLEEP_TAG:-}
mkdir -p $O
T="timeout -k 10"
for sl in ${SLEEPS:-0 1 2 4 -3 -6}; do
for a in "--stencil 100 --points 27" "--stencil 100 --points 7" ""; do
  tag=s$sl$(echo "x$a" | tr -d ' -')
  SBLAS_TRSV_SLEEP=$sl $T 300 python s-blas_amd/tools/bench_sptrsv.py $a --steps 5 > $O/trsv_$tag.json 2> $O/trsv_$tag.err || { tail -20 $O/trsv_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsv_$tag.json'))
print('$tag', {k: v['ms'] for k, v in d['executors'].items() if k.startswith('pull')})"
done
done
echo done
