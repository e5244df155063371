#!/bin/bash
# round 5: pull SpTRSV defaults 128 / 64 threads per workgroup (natural /
# level order): the SpTRSV / SpTRSM tests, the stand-in and stencil timings,
# and the default bench line (config5 leg) -> profiles/r05/trsv_waves/
set -o pipefail
O=gpurun_out/r05_trsv3
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cli_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -k "trsv or trsm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for A in "" "--stencil 100 --points 27" "--stencil 100 --points 7"; do
  $T 150 python s-blas_amd/tools/bench_sptrsv.py --steps 5 --no-cpu-baseline $A --mgpu 4 >> $O/sptrsv.jsonl 2>> $O/sptrsv.err || { tail -5 $O/sptrsv.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/sptrsv.jsonl'):
    d=json.loads(l); print(d['data'][:40], {k: v['ms'] for k, v in d['executors'].items()})"
$T 400 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); c=d['config5']
print(d['value'], d['roofline']['frac'], c['ms'], c['exact'] if 'exact' in c else c.get('check'), c.get('blocks4'))"
