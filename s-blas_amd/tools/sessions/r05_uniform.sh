#!/bin/bash
# round 5, after the generator fix (profiles/r05/gen/): the default bench line,
# the ctx driver's N = 1 line, rank slices (N = 8 / 4 floor + xsort), configs[2]
# per-rank CSR5 under the nnz and cost-weighted splits -> profiles/r05/uniform/
set -o pipefail
O=gpurun_out/r05_uniform
mkdir -p $O
T="timeout -k 10"
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
$T 300 python bench.py --driver ctx --no-cpu-baseline > $O/bench_ctx1.json 2> $O/bench_ctx1.err || { tail -20 $O/bench_ctx1.err; exit 1; }
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 8,4,2 --ranks 0 --algos xsort,csr5,rowsplit --floor --reps 10 > $O/slices.jsonl 2> $O/slices.err || { tail -20 $O/slices.err; exit 1; }
$T 400 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --partition nnz --ranks all --algos csr5 --reps 8 > $O/c3_nnz.jsonl 2> $O/c3_nnz.err || { tail -20 $O/c3_nnz.err; exit 1; }
for w in 0 6 12; do
  $T 400 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --partition cost --row-cost $w --ranks all --algos csr5 --reps 8 > $O/c3_cost$w.jsonl 2> $O/c3_cost$w.err || { tail -20 $O/c3_cost$w.err; exit 1; }
done
python3 - <<'PY'
import json, glob
O = "gpurun_out/r05_uniform"
d = json.loads(open(f"{O}/bench_default.json").read().strip().splitlines()[-1])
print("default", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["measured_peak"]["read_GBps"], d["rowsplit_beside"]["kernel_ms"], d["config3"]["kernel_ms_max"], d["config4"]["kernel_ms_max"], d["config5"]["ms"], d["config5"]["levels"], d["config5"]["blocks4"]["ms"])
e = json.loads(open(f"{O}/bench_ctx1.json").read().strip().splitlines()[-1])
print("ctx", e["value"], e["ms_per_step"], e["config3"]["kernel_ms_max"])
for line in open(f"{O}/slices.jsonl"):
    x = json.loads(line)
    print("floor" if "floor" in x else x["algo"], x["world"], x.get("us", x.get("cold_span_us")))
for f in [f"{O}/c3_nnz.jsonl"] + sorted(glob.glob(f"{O}/c3_cost*.jsonl")):
    rows = [json.loads(l) for l in open(f)]
    for w in (8, 4):
        r = [x for x in rows if x["world"] == w]
        print(f.split("/")[-1], w, "max", max(x["cold_span_us"] for x in r), [x["cold_span_us"] for x in r])
PY
