# round 3: what bounds the N = 8 slice -- timing modes of the default (dynamic, one-chunk) kernel:
# 0 product, 8 no x gathers, 9 no gathers + plain LDS stores (wrong y: timing only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_modes
mkdir -p $O
rc=0
for md in 0 8 9; do
  SBLAS_XS_MODE=$md timeout -k 10 240 python3 s-blas_amd/tools/bench_slice.py --worlds 1,4,8 --algos xsort > $O/mode_$md.jsonl 2> $O/e_$md.err || { rc=$?; break; }
  echo "mode $md"; cat $O/mode_$md.jsonl
done
echo rc=$rc
