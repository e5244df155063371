#!/bin/bash
# round 4: overlapped ctx exchange (sblas_ctx_matrix_upload_parts), loopback parity
set -o pipefail
O=gpurun_out/r04_overlap; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_ctx_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
