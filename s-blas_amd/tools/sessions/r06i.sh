# r06i: the torchrun rehearsals (topology keys) and the ctx / peer tests after the registry change
set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_ctx_gpu.py tests/test_bench_gpu.py > gpurun_out/r06i/tests.log 2>&1
