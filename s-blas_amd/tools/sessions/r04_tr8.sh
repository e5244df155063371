#!/bin/bash
# round 4: torchrun 8 ranks (gloo) on one GPU at full config-2 size, both legs checked
set -o pipefail
O=gpurun_out/r04_tr8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread "tests/test_cli_gpu.py::test_torchrun_8_ranks_full_size" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
