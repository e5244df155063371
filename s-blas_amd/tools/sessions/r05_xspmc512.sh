#!/bin/bash
# round 5: xsort counters on the 512-thread default (uniform config 2 and the
# 27-point stencil, cold launches) -> profiles/r05/xspmc512/
set -o pipefail
O=gpurun_out/r05_xspmc512
mkdir -p $O
bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmv_xsort" $O/n1 s-blas_amd/tools/spmv_one.py --algo xsort --reps 4 --cold --scrub read || exit 1
bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmv_xsort" $O/s27 s-blas_amd/tools/spmv_one.py --matrix stencil27 --grid 128 --algo xsort --reps 4 --cold --scrub read || exit 1
cat $O/n1/summary.json $O/s27/summary.json
