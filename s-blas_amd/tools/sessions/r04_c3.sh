#!/bin/bash
# round 4: configs[2] leg on every bench line (ctx + torch paths), CPU baseline pinning
set -o pipefail
O=gpurun_out/r04_c3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_bench_gpu.py "tests/test_cli_gpu.py::test_config3_two_ranks" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -50 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail -30 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --driver ctx > $O/bench_ctx1.json 2> $O/bench_ctx1.err || { echo CTX FAILED; tail -30 $O/bench_ctx1.err; exit 1; }
tail -5 $O/tests.log; cat $O/bench_default.json $O/bench_ctx1.json | cut -c1-600
