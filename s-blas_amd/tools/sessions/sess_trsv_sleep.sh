#!/bin/bash
# SpTRSV pull executor: poll back-off sweep (SBLAS_TRSV_SLEEP), config 5 stand-in
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for v in 1 0 4 16 64 -3 -5 -7 1; do
  SBLAS_TRSV_SLEEP=$v $T 240 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 5 > gpurun_out/btrsv.log 2>&1 || { tail -5 gpurun_out/btrsv.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/btrsv.log") if l.startswith("{")][-1])
r = d["executors"]
p = {k: r[k] for k in ("pull_csr", "pull_level_order") if k in r}
print("SBLAS_TRSV_SLEEP=" + sys.argv[1], {k: (v["ms"], v["rel_l1_vs_xref"]) for k, v in p.items()}, flush=True)
PY
done
