# r06m: the full -m gpu suite and smoke() on the current tree
set -o pipefail
mkdir -p gpurun_out/r06m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06m/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06m/smoke.log 2>&1 || exit 1
