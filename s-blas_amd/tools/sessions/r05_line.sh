#!/bin/bash
# round 5: the default bench line and a 2-rank launcher rehearsal (gloo, one
# GPU) whose line carries config4.grid -> profiles/r05/line/
set -o pipefail
O=gpurun_out/r05_line
mkdir -p $O
T="timeout -k 10"
$T 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
$T 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err || { tail -20 $O/bench_2rank_gloo.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_line"
d = json.loads(open(f"{O}/bench_default.json").read().strip().splitlines()[-1])
print("N=1", d["value"], d["roofline"], d["config3"]["kernel_ms_max"], d["config4"]["kernel_ms_max"], d["config5"]["ms"], d["config5"]["blocks4"]["ms"], d["traffic_source"])
e = json.loads(open(f"{O}/bench_2rank_gloo.json").read().strip().splitlines()[-1])
print("N=2", e["value"], e["config4"]["kernel_ms_max"], e["config4"]["check"], e["config4"]["grid"])
PY
