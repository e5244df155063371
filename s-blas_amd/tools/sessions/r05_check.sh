#!/bin/bash
# round 5: full -m gpu suite + smoke after the uniform-matrix retune, then the
# default bench line and the N = 1..8 slices -> profiles/r05/retune/
set -o pipefail
O=gpurun_out/r05_check
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --ranks 0 --algos xsort --reps 8 > $O/slices.jsonl 2> $O/slices.err || { tail -20 $O/slices.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_check"
d = json.loads(open(f"{O}/bench_default.json").read().strip().splitlines()[-1])
print("default", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["measured_peak"]["read_GBps"], d["rowsplit_beside"]["kernel_ms"], d["config3"]["kernel_ms_max"], d["config4"]["kernel_ms_max"], d["config5"]["ms"])
for line in open(f"{O}/slices.jsonl"):
    x = json.loads(line); print(x["world"], x["algo"], x["cold_span_us"])
PY
