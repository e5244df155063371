#!/bin/bash
# round 5: why CSR5 pays ~50 us per M rows on short rows -- counters of the
# plain CSR5 tile (SBLAS_CSR5_PANEL=0) on configs[2]'s N = 8 nnz-split heavy
# rank (0: 52k rows x 96) and light rank (7: 552k rows x 9), same entry count
# -> profiles/r05/c5light/
set -o pipefail
O=gpurun_out/r05_c5light
mkdir -p $O
export SBLAS_CSR5_PANEL=0
for r in 7; do
  bash s-blas_amd/tools/prof_counters_cmd.sh "k_spmv_csr5<true, 2>" $O/rank$r s-blas_amd/tools/bench_slice.py --worlds 8 --partition nnz --ranks $r --algos csr5 --reps 4 || exit 1
done
timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 8 --partition nnz --ranks 0,7 --algos csr5 --reps 8 > $O/spans_plain.jsonl 2> $O/spans.err || { tail -5 $O/spans.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_c5light"
a = json.load(open(f"{O}/rank0/summary.json")); b = json.load(open(f"{O}/rank7/summary.json"))
for k in sorted(set(a) | set(b)):
    print(f"{k:40s} {a.get(k, float('nan')):16.1f} {b.get(k, float('nan')):16.1f}")
PY
cat $O/spans_plain.jsonl
timeout -k 10 300 python s-blas_amd/tools/bench_spmm_slices.py --split cols --worlds 1,2,4,8 > $O/spmm_slices_cols.jsonl 2> $O/spmm_cols.err || { tail -20 $O/spmm_cols.err; exit 1; }
grep summary $O/spmm_slices_cols.jsonl
