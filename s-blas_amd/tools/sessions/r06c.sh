# r06c: deterministic-mode tests after the shared-turn fix
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_configs_gpu.py -k "deterministic or rank_slice or xsort" tests/test_spmv_gpu.py > gpurun_out/r06c/tests.log 2>&1
