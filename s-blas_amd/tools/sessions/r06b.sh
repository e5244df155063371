# r06b: full GPU suite on the cleaned library, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r06b/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r06b/bench.json 2> gpurun_out/r06b/bench.err
