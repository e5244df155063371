#!/bin/bash
# round 5: counters of the read probe (one span per workgroup, nt, 2 / CU)
# to compare its L1 -> L2 requests in flight with xsort's ~97 per CU
# -> profiles/r05/probepmc/
set -o pipefail
O=gpurun_out/r05_probepmc
mkdir -p $O
timeout -k 10 60 python s-blas_amd/tools/probe_one.py --mode 4 --wg 2 > $O/run.txt 2>&1 || { cat $O/run.txt; exit 1; }
cat $O/run.txt
bash s-blas_amd/tools/prof_counters_cmd.sh "k_probe_read" $O/nt2 s-blas_amd/tools/probe_one.py --mode 4 --wg 2 --reps 2 || exit 1
bash s-blas_amd/tools/prof_counters_cmd.sh "k_probe_read" $O/plain16 s-blas_amd/tools/probe_one.py --mode 3 --wg 16 --reps 2 || exit 1
