# round 3: per-workgroup timeline of the N = 8 slice (persistent xsort kernel)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trace
mkdir -p $O
SBLAS_XS_BATCH=0 SBLAS_XS_TRACE=$O/trace8.txt timeout -k 10 300 python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort --reps 2 > $O/slice8.jsonl 2> $O/e1.err &&
SBLAS_XS_TRACE=$O/trace1.txt timeout -k 10 300 python3 s-blas_amd/tools/bench_slice.py --worlds 1 --algos xsort --reps 2 > $O/slice1.jsonl 2> $O/e3.err
echo rc=$?
wc -l $O/*.txt
