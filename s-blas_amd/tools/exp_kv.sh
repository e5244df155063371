set -o pipefail
for KV in 1 0; do for M in 0 2; do
  echo -n "kv $KV mode $M: "; SBLAS_XS_KV=$KV SBLAS_XS_MODE=$M timeout -k 5 60 python3 s-blas_amd/tools/spmv_one.py --reps 20 2>/dev/null | tail -1 || exit 1
done; done
echo -n "kv 1 cold: "; timeout -k 5 60 python3 s-blas_amd/tools/spmv_one.py --reps 20 --cold 2>/dev/null | tail -1
