#!/bin/bash
# round 4: the default bench line's config3 leg, three runs back to back
set -o pipefail
O=gpurun_out/r04_c3check; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$i.json 2>>$O/err.log || exit 1
  tail -1 $O/bench_$i.json | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print($i, d['ms_per_step'], d['rowsplit_beside']['kernel_ms'], d['config3']['kernel_ms_max'], d['config3']['roofline']['frac'])"
done
