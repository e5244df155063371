# round 3: planner knobs on rank slices (items per slot, wide-entry budget)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_slice_plan
mkdir -p $O
rc=0
for v in "SBLAS_XS_K=2" "SBLAS_XS_WBUDGET=0.5" "SBLAS_XS_WBUDGET=0.6" "SBLAS_XS_WBUDGET=0.7" "SBLAS_XS_WBUDGET=0.85" "SBLAS_XS_MODE=0"; do
  env $v timeout -k 10 240 python3 s-blas_amd/tools/bench_slice.py --worlds 2,4,8 --algos xsort > $O/$v.jsonl 2> $O/$v.err || { rc=$?; break; }
  echo "$v"; cat $O/$v.jsonl | cut -c1-160
done
echo rc=$rc
