# r06u: the overlapped exchange's kernel side at N = 2 / 4 (rank 0's cyclic slice whole vs in 2 / 3 parts back to back, cold)
set -o pipefail
mkdir -p gpurun_out/r06u
timeout -k 10 500 python -u s-blas_amd/tools/bench_slice.py --worlds 2,4 --algos xsort --parts 2 --reps 10 > gpurun_out/r06u/parts2.jsonl 2> gpurun_out/r06u/err.log || exit 1
timeout -k 10 500 python -u s-blas_amd/tools/bench_slice.py --worlds 2,4 --algos xsort --parts 3 --reps 10 > gpurun_out/r06u/parts3.jsonl 2>> gpurun_out/r06u/err.log || exit 1
