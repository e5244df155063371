#!/bin/bash
# round 4: full-size config tests incl. every CSR5 / row-split form and the panel choice
set -o pipefail
O=gpurun_out/r04_cfgtests; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_configs_gpu.py tests/test_spmv_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
