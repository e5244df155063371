# round 3: the ctx driver with N > 1 ranks on one GPU (SBLAS_CTX_LOOPBACK) -- the N > 1 logic of
# sblas_ctx and bench.py's ctx path, checked against the oracle
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_loopback
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ctx_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
timeout -k 10 300 python bench.py --gpus 8 --ctx-loopback --check --no-cpu-baseline > $O/bench_loopback8.json 2> $O/b8.err
echo rc=$rc $?
head -c 1500 $O/bench_loopback8.json
