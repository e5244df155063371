set -o pipefail
R="timeout -k 5 60 python3 s-blas_amd/tools/spmv_one.py --reps 20"
echo -n "warm: "; $R 2>/dev/null | tail -1 || exit 1
echo -n "cold write-scrub: "; $R --cold 2>/dev/null | tail -1 || exit 1
echo -n "cold read-scrub: "; $R --cold --scrub read 2>/dev/null | tail -1 || exit 1
for Q in 1 2 4; do for L in 0.5 1.0 1.5; do
  echo -n "q $Q lambda $L cold-read: "; SBLAS_XS_Q=$Q SBLAS_XS_LAMBDA=$L $R --cold --scrub read 2>/dev/null | tail -1 || exit 1
done; done
for W in 0.5 0.7 0.85; do
  echo -n "wbudget $W cold-read: "; SBLAS_XS_WBUDGET=$W $R --cold --scrub read 2>/dev/null | tail -1 || exit 1
done
