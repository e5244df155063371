#!/bin/bash
# FETCH/WRITE and L2 hit/miss of the SpMM C-tile kernels on config 4 (separate passes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/pmc_spmm
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  d=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$d -o run --output-format csv -- python3 s-blas_amd/tools/bench_spmm.py --no-cpu-baseline --steps 5 > $O.$d.log 2>&1 || { tail -5 $O.$d.log; exit 1; }
done
echo done
