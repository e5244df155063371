#!/bin/bash
# round 5: counters of xsort on the 27-point stencil stand-in (the structured
# leg's matrix, cold launches) -> profiles/r05/s27pmc/
set -o pipefail
O=gpurun_out/r05_s27pmc
mkdir -p $O
bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmv_xsort" $O/s27 s-blas_amd/tools/spmv_one.py --matrix stencil27 --grid 128 --algo xsort --reps 4 --cold --scrub read || exit 1
cat $O/s27/summary.json | head -40
