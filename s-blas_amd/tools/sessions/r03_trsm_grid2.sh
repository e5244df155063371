# SpTRSM pull at the default V: workgroups per CU 1 / 2 / 4 at rhs 16..64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsm_grid2
mkdir -p $O
T="timeout -k 10"
for w in 1 2 4; do
for a in "--stencil 100 --points 27" ""; do
  tag=w$w$(echo "x$a" | tr -d ' -')
  SBLAS_TRSM_WG_PER_CU=$w $T 500 python s-blas_amd/tools/bench_sptrsv.py $a --rhs 8,16,32,64 --no-push-rhs --steps 3 > $O/trsm_$tag.json 2> $O/trsm_$tag.err || { tail -20 $O/trsm_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trsm_$tag.json'))
print('$tag', {k.replace('trsm_pull_',''): v['ms'] for k, v in d['executors'].items() if 'auto_rhs' in k})"
done
done
echo done
