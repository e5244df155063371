#!/bin/bash
# round 5: where xsort's R-MAT time goes (structured leg's 0.39): plan,
# item timeline (1024-thread trace twin), counters -> profiles/r05/rmat/
set -o pipefail
O=gpurun_out/r05_rmat
mkdir -p $O
T="timeout -k 10 200"
SBLAS_XS_TIMING=1 $T python s-blas_amd/tools/spmv_one.py --matrix rmat --scale 21 --algo xsort --reps 8 --cold --scrub read > $O/plan.txt 2>&1 || { tail -5 $O/plan.txt; exit 1; }
grep -v amdgpu.ids $O/plan.txt
SBLAS_XS_TRACE=$O/trace.txt $T python s-blas_amd/tools/spmv_one.py --matrix rmat --scale 21 --algo xsort --reps 3 --cold --scrub read > $O/trace_run.txt 2>&1 || { tail -5 $O/trace_run.txt; exit 1; }
python3 s-blas_amd/tools/xs_trace.py $O/trace.txt > $O/trace_summary.txt && cat $O/trace_summary.txt
SBLAS_XS_TRACE=$O/trace_c2.txt $T python s-blas_amd/tools/spmv_one.py --algo xsort --reps 3 --cold --scrub read > $O/trace_c2_run.txt 2>&1 || { tail -5 $O/trace_c2_run.txt; exit 1; }
python3 s-blas_amd/tools/xs_trace.py $O/trace_c2.txt > $O/trace_c2_summary.txt && cat $O/trace_c2_summary.txt
rm -f $O/trace.txt $O/trace_c2.txt
bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmv_xsort" $O/pmc s-blas_amd/tools/spmv_one.py --matrix rmat --scale 21 --algo xsort --reps 4 --cold --scrub read > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
