# SpTRSV pull executor: polls in flight per lane (SBLAS_TRSV_PIPE = 1..4)
# parity (KATs, config 5 exact) and config-5 timing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsv_pipe
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "pipelined or pipe or pull_backoff" \
    tests/test_kernels_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in 1 2 3 4 1 2 3 4; do
  SBLAS_TRSV_PIPE=$p $T 300 python s-blas_amd/tools/bench_sptrsv.py --no-cpu-baseline --steps 5 > $O/bench_pipe$p.json 2> $O/bench_pipe$p.err || { tail -20 $O/bench_pipe$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_pipe$p.json')); print('pipe $p', {k: v for k, v in d.items() if 'ms' in k or 'pull' in k})"
done
echo done
