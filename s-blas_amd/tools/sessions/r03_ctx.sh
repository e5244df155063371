# round 3: ctx driver (allreduce exchange, timing protocol), bench --driver ctx, SpMM per-handle scratch
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_ctx
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ctx_gpu.py tests/test_bench_gpu.py "tests/test_kernels_gpu.py::test_spmm_two_handles_two_streams" > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --driver ctx --no-cpu-baseline > $O/bench_ctx_xsort.json 2> $O/bench_ctx_xsort.err &&
timeout -k 10 300 python bench.py --gpus 1 --driver ctx --algo csr5 --exchange allreduce --no-cpu-baseline > $O/bench_ctx_csr5_allreduce.json 2> $O/bench_ctx_csr5.err &&
timeout -k 10 300 ./s-blas_amd/bin/spmv_ctx 1 2000000 2 1 10 1 > $O/spmv_ctx_cfg3.log 2>&1
echo rc=$?
tail -3 $O/tests.log
