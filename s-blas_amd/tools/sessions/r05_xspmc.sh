#!/bin/bash
# round 5: counters of the xsort kernel on the uniform config 2 (cold launches)
# -> profiles/r05/xspmc/
set -o pipefail
O=gpurun_out/r05_xspmc
mkdir -p $O
bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmv_xsort" $O/n1 s-blas_amd/tools/spmv_one.py --algo xsort --reps 4 --cold --scrub read || exit 1
cat $O/n1/summary.json
