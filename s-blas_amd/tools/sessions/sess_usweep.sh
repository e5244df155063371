#!/bin/bash
# chunks per dynamic claim (U) per slice size: U=1 vs U=2 at N = 1, 2, 4, 8 (rank 0's cyclic slice)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/usweep.jsonl
for u in 1 2; do
  echo "== SBLAS_XS_U=$u" >> gpurun_out/usweep.jsonl
  SBLAS_XS_U=$u $T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort >> gpurun_out/usweep.jsonl 2>&1 || { tail -5 gpurun_out/usweep.jsonl; exit 1; }
done
echo "== planner default" >> gpurun_out/usweep.jsonl
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos xsort >> gpurun_out/usweep.jsonl 2>&1 || { tail -5 gpurun_out/usweep.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/usweep.jsonl
