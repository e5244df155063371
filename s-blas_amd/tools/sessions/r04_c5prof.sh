#!/bin/bash
# round 4: kernel breakdown of the panel CSR5 on config 2 (and its light/heavy parts)
set -o pipefail
O=gpurun_out/r04_c5prof; mkdir -p $O
export TMPDIR=/tmp
for P in full light heavy; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$P -o run --output-format csv -- python3 s-blas_amd/tools/exp_split.py --parts $P --variants csr5 --reps 6 > $O/$P.log 2>&1 || { tail -5 $O/$P.log; exit 1; }
  echo "== $P"; grep -E "csr5|panel" $O/$P/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
