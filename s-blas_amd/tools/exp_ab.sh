# A/B of two libsblas builds on one box: alternating runs, cold read-scrub and warm
set -o pipefail
R="timeout -k 5 60 python3 s-blas_amd/tools/spmv_one.py --reps 30"
for i in 1 2 3; do
  echo -n "new  cold-read: "; $R --cold --scrub read 2>/dev/null | tail -1 || exit 1
  echo -n "prev cold-read: "; SBLAS_LIB=s-blas_amd/ab/libsblas_prev.so $R --cold --scrub read 2>/dev/null | tail -1 || exit 1
  echo -n "new  warm: "; $R 2>/dev/null | tail -1 || exit 1
  echo -n "prev warm: "; SBLAS_LIB=s-blas_amd/ab/libsblas_prev.so $R 2>/dev/null | tail -1 || exit 1
done
