#!/bin/bash
# counters of the MSD transpose kernels (per-mode summaries are made from the merged output)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/pmc_tr2
bash s-blas_amd/tools/prof_cmd.sh k_rx2_scatter $O s-blas_amd/tools/bench_transpose.py --mgpu= --steps 3 > gpurun_out/pmc_tr2.txt 2>&1 || { tail -5 gpurun_out/pmc_tr2.txt; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 s-blas_amd/tools/bench_transpose.py --mgpu= --steps 3 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
echo done
