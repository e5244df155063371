#!/bin/bash
# SpTRSV pull executor confined to fewer XCDs (SBLAS_TRSV_XCDS) x workgroups per CU
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for v in "SBLAS_TRSV_XCDS=8" "SBLAS_TRSV_XCDS=1" "SBLAS_TRSV_XCDS=1 SBLAS_TRSV_WG_PER_CU=2" "SBLAS_TRSV_XCDS=1 SBLAS_TRSV_WG_PER_CU=4" "SBLAS_TRSV_XCDS=2" "SBLAS_TRSV_XCDS=4" "SBLAS_TRSV_XCDS=2 SBLAS_TRSV_WG_PER_CU=2"; do
  env $v $T 240 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 5 > gpurun_out/btrsv.log 2>&1 || { tail -5 gpurun_out/btrsv.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/btrsv.log") if l.startswith("{")][-1])
r = d["executors"]
p = {k: r[k] for k in ("pull_csr", "pull_level_order") if k in r}
print(sys.argv[1], {k: (v["ms"], v["rel_l1_vs_xref"]) for k, v in p.items()})
PY
done
