#!/bin/bash
# round 5: N = 8 slice streaming floor and configs[2]'s
# per-rank CSR5 slices under the nnz split and the cost-weighted split (item 2)
# -> profiles/r05/slice_floor/, profiles/r05/c3cost/
set -o pipefail
O=gpurun_out/r05_slice
mkdir -p $O
T="timeout -k 10"
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --ranks 0 --algos xsort --floor --reps 10 > $O/floor_w8_w4.jsonl 2> $O/floor.err || { tail -20 $O/floor.err; exit 1; }
$T 400 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --partition nnz --ranks all --algos csr5 --reps 8 > $O/c3_nnz.jsonl 2> $O/c3_nnz.err || { tail -20 $O/c3_nnz.err; exit 1; }
for w in 4 6 8; do
  $T 400 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --partition cost --row-cost $w --ranks all --algos csr5 --reps 8 > $O/c3_cost$w.jsonl 2> $O/c3_cost$w.err || { tail -20 $O/c3_cost$w.err; exit 1; }
done
python3 - <<'PY'
import json, glob
O = "gpurun_out/r05_slice"
for line in open(f"{O}/floor_w8_w4.jsonl"):
    d = json.loads(line)
    if "floor" in d:
        print("floor", d["world"], d["us"], d["best_shape"], d["bytes"], d["gbps"])
    else:
        print("xsort", d["world"], d["rank"], d["cold_span_us"], d["warm_us"])
for f in [f"{O}/c3_nnz.jsonl"] + sorted(glob.glob(f"{O}/c3_cost*.jsonl")):
    rows = [json.loads(l) for l in open(f)]
    for w in (8, 4):
        r = [x for x in rows if x["world"] == w]
        print(f.split("/")[-1], w, "max", max(x["cold_span_us"] for x in r), [x["cold_span_us"] for x in r], [x["local_nnz"] for x in r])
PY
$T 300 python s-blas_amd/tools/bench_spmm_slices.py --worlds 1,2,4,8 > $O/spmm_slices.jsonl 2> $O/spmm_slices.err || { tail -20 $O/spmm_slices.err; exit 1; }
grep summary $O/spmm_slices.jsonl
