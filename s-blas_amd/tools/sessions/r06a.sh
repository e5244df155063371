set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "block_devices or peer_refusal or persistent_handle" tests/test_ctx_gpu.py::test_ctx_two_contexts_peer_refcount tests/test_ctx_gpu.py::test_ctx_comm_info_rccl tests/test_bench_gpu.py > gpurun_out/r06a/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
