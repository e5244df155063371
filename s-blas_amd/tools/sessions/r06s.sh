# r06s: CSR -> CSC transpose on config 2 (single device + multi-block compose), rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out/r06s
export TMPDIR=/tmp
timeout -k 10 300 python -u s-blas_amd/tools/bench_transpose.py --mgpu 1,2,4 > gpurun_out/r06s/transpose.jsonl 2> gpurun_out/r06s/err.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06s/prof -o run --output-format csv -- python3 s-blas_amd/tools/bench_transpose.py --mgpu 1 > gpurun_out/r06s/transpose_prof.jsonl 2>> gpurun_out/r06s/err.log || exit 1
