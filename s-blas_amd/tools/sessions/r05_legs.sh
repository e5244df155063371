#!/bin/bash
# round 5: the default bench line with the config4 / config5 legs, the probe
# ceiling and the thread-swept CPU baseline; the ctx driver's N = 1 line;
# stencil27 xsort with 1 GiB and 4 GiB cold sweeps (profiles/r05/legs/)
set -o pipefail
O=gpurun_out/r05_legs
mkdir -p $O
T="timeout -k 10"
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
$T 300 python bench.py --driver ctx --no-cpu-baseline > $O/bench_ctx1.json 2> $O/bench_ctx1.err || { tail -20 $O/bench_ctx1.err; exit 1; }
for g in 1 4; do
  $T 300 python bench.py --matrix stencil27 --algo xsort --scrub-gib $g --no-cpu-baseline --no-config3 --no-config4 --no-config5 --no-rowsplit-beside > $O/stencil27_xsort_scrub${g}.json 2> $O/stencil27_scrub${g}.err || { tail -20 $O/stencil27_scrub${g}.err; exit 1; }
done
python3 - <<'PY'
import json
O="gpurun_out/r05_legs"
d=json.loads(open(f"{O}/bench_default.json").read().strip().splitlines()[-1])
print("default", d["value"], d["ms_per_step"], d["roofline"], d.get("measured_peak"))
print("config4", json.dumps(d.get("config4"))[:600])
print("config5", json.dumps(d.get("config5"))[:900])
print("cpu", d["cpu_baseline"].get("thread_sweep_gflops"), d["cpu_baseline"].get("value"), d["cpu_baseline"].get("cgroup_cpu_quota"))
for g in (1, 4):
    s=json.loads(open(f"{O}/stencil27_xsort_scrub{g}.json").read().strip().splitlines()[-1])
    print("stencil27 scrub", g, s["ms_per_step"], s["roofline"]["achieved"], s["roofline"]["frac"], s.get("measured_peak", {}).get("read_GBps"))
PY
