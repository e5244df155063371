#!/bin/bash
# N=8 slice diagnostics (xsort experiment modes) + default bench line with the measured copy peak
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/slicediag.jsonl
for v in "SBLAS_XS_MODE=0" "SBLAS_XS_MODE=2" "SBLAS_XS_MODE=1" "SBLAS_XS_U=1" "SBLAS_XS_U=3" "SBLAS_XS_NOWIDE=1" "SBLAS_XS_ROWS=4096"; do
  echo "== $v" >> gpurun_out/slicediag.jsonl
  env $v $T 200 python s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort >> gpurun_out/slicediag.jsonl 2>&1 || { tail -5 gpurun_out/slicediag.jsonl; exit 1; }
done
grep -v amdgpu.ids gpurun_out/slicediag.jsonl
$T 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
