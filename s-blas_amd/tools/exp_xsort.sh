#!/bin/bash
# xsort timing experiments: kernel-only times of the
# column-sorted SpMV under the SBLAS_XS_* knobs, config-2 matrix.
set -o pipefail
O=gpurun_out/xs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "${@:-BASE=1}"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 200 python bench.py --algo xsort --cache warm --no-cpu-baseline --steps 10 --warmup 2 \
    > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $v"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); print('%-40s kernel %.1f us  step %.1f us  frac %.3f' % ('$v', d['kernel_ms']*1e3, d['ms_per_step']*1e3, d['roofline']['frac']))"
done
