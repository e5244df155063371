#!/bin/bash
# xsort parity after the claim change, then the headline evidence (sess_headline.sh)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "xsort or config2 or config3" > gpurun_out/t_xs.log 2>&1 || { tail -30 gpurun_out/t_xs.log; exit 1; }
tail -1 gpurun_out/t_xs.log
bash s-blas_amd/tools/sessions/sess_headline.sh
