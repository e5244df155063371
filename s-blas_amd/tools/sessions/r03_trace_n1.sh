# per-workgroup timeline of the default xsort launch at N = 1 (SBLAS_XS_TRACE):
# per-XCD entry / exit, to size any XCD-aware rebalancing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trace_n1
mkdir -p $O
rm -f $O/trace.txt
SBLAS_XS_TRACE=$O/trace.txt timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort --reps 3 > $O/slice.jsonl 2> $O/slice.err || { tail -20 $O/slice.err; exit 1; }
wc -l $O/trace.txt
echo done
