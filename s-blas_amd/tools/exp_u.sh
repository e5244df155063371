set -o pipefail
for M in 0 2 4 6; do for U in 1 2 3 4; do
  echo -n "mode $M U $U: "; SBLAS_XS_MODE=$M SBLAS_XS_U=$U timeout -k 5 60 python3 s-blas_amd/tools/spmv_one.py --reps 20 2>/dev/null | tail -1 || exit 1
done; done
