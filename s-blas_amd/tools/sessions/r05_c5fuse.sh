#!/bin/bash
# round 5: CSR5 panel form with calibrate + reduce fused (k_c5_panel_reduce):
# CSR5 tests (incl. fused vs separate bit-identity), then config 2 CSR5 cold at
# N = 1 and configs[2]'s N = 8 cost-split slices, fused vs SBLAS_C5_FUSE=0
# -> profiles/r05/c5fuse/
set -o pipefail
O=gpurun_out/r05_c5fuse
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py tests/test_ctx_gpu.py -x -q --timeout 200 --timeout-method thread -k "csr5 or config3 or c5" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for f in 1 0; do
    SBLAS_C5_FUSE=$f $T 300 python s-blas_amd/tools/bench_slice.py --worlds 1 --ranks 0 --algos csr5 --reps 8 > $O/n1_f${f}_$r.jsonl 2> $O/n1_f${f}_$r.err || { tail -5 $O/n1_f${f}_$r.err; exit 1; }
    SBLAS_C5_FUSE=$f $T 300 python s-blas_amd/tools/bench_slice.py --worlds 8 --ranks all --algos csr5 --partition cost --reps 8 > $O/n8_f${f}_$r.jsonl 2> $O/n8_f${f}_$r.err || { tail -5 $O/n8_f${f}_$r.err; exit 1; }
    python3 - "$O" "$f" "$r" <<'PY'
import json, sys
O, f, r = sys.argv[1:]
a = [json.loads(l) for l in open(f"{O}/n1_f{f}_{r}.jsonl")]
b = [json.loads(l) for l in open(f"{O}/n8_f{f}_{r}.jsonl")]
print("fuse", f, "run", r, "N=1", a[0]["cold_span_us"], "N=8 max", max(x["cold_span_us"] for x in b if "cold_span_us" in x))
PY
  done
done
