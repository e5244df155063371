#!/bin/bash
# full -m gpu suite + smoke on the round-4 end tree (profiles/r04/end/)
set -o pipefail
O=gpurun_out/r04_end
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --driver ctx > $O/bench_ctx1_alias.json 2> $O/bench_ctx1_alias.err || { tail -20 $O/bench_ctx1_alias.err; exit 1; }
tail -1 $O/bench_ctx1_alias.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['config3']['roofline']['frac'])"
