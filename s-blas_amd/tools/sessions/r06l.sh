# r06l: SpMM C tile, pipelined stream loads with / without epoch-synchronised sibling row blocks (config 4)
set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "spmm" -m gpu > gpurun_out/r06l/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u s-blas_amd/tools/exp_spmm.py --rounds 2 --opts '[{}, {"spmm_pipe": 1}, {"spmm_pipe": 1, "spmm_epochs": 4}, {"spmm_pipe": 1, "spmm_epochs": 8}, {"spmm_pipe": 1, "spmm_epochs": 16}, {"spmm_pipe": 1, "spmm_epochs": 16, "spmm_lag": 2}, {"spmm_pipe": 1, "spmm_epochs": 32, "spmm_lag": 2}]' > gpurun_out/r06l/spmm.jsonl 2> gpurun_out/r06l/err.log || exit 1
