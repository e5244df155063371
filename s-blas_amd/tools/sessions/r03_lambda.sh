# round 3: planner cost-model sweep on rank slices (lambda = per-x-line cost)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_lambda
mkdir -p $O
rc=0
for lam in 1.0 1.5 2.0 3.0 5.0; do
  SBLAS_XS_BATCH=0 SBLAS_XS_LAMBDA=$lam timeout -k 10 240 python3 s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort > $O/lam_$lam.jsonl 2> $O/e_$lam.err || { rc=$?; break; }
  echo "lambda $lam"; cat $O/lam_$lam.jsonl
done
echo rc=$rc
