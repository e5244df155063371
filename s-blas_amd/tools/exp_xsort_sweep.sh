#!/bin/bash
# xsort planner-knob sweep on config 2 (kernel ms cold, warm), each variant
# under its own timeout; usage: bash exp_xsort_sweep.sh "name:ENV=V,ENV=V" ...
set -o pipefail
mkdir -p gpurun_out/sw
for spec in "$@"; do
  n=${spec%%:*}; e=${spec#*:}; e=${e//,/ }
  env $e timeout -k 10 120 python bench.py --algo xsort --no-cpu-baseline --steps 20 > gpurun_out/sw/$n.log 2>&1 || { echo "$n failed"; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/sw/$n.log') if l.startswith('{')][0]); print('$n', d['kernel_ms'], d['warm']['kernel_ms'])"
done
