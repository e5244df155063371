#!/bin/bash
# round-end evidence: full GPU suite, smoke, default bench line, rocprofv3
# kernel-trace stats of the same bench command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
$T 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py > gpurun_out/bench_under_rocprof.json 2> gpurun_out/prof.err || { tail -20 gpurun_out/prof.err; exit 1; }
cat gpurun_out/bench_under_rocprof.json
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
