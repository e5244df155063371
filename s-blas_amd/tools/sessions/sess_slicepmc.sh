#!/bin/bash
# N = 8 per-rank slice (rank 0's cyclic share of config 2), xsort: FETCH/WRITE
# passes and the prof_cmd.sh counter groups, each pass its own bounded run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/pmc_slice8
B="s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort --reps 10"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 $B > $O.$c.log 2>&1 || { tail -5 $O.$c.log; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O.trace.log 2>&1 || { tail -5 $O.trace.log; exit 1; }
bash s-blas_amd/tools/prof_cmd.sh k_spmv_xsort $O/groups $B > $O.groups.log 2>&1 || { tail -5 $O.groups.log; exit 1; }
tail -3 $O.groups.log
echo done
