#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the transpose kernels (separate passes), per kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/pmc_tr3
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 s-blas_amd/tools/bench_transpose.py --mgpu= --steps 3 > $O.$c.log 2>&1 || { tail -5 $O.$c.log; exit 1; }
done
for k in "k_rx2_scatter<256, 0" "k_rx2_scatter<256, 1" "k_rx2_scatter<256, 2" "k_rx2_count<0>" "k_rx2_count<1>"; do
  python3 s-blas_amd/tools/pmc_traffic.py --kernel "$k" --fetch $O/FETCH_SIZE --write $O/WRITE_SIZE --out /tmp/pt.json > /dev/null 2>&1 || { echo "parse failed for $k"; continue; }
  echo "$k $(cat /tmp/pt.json)"
done
