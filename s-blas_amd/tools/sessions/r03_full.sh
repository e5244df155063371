# round 3: the full -m gpu suite (as the driver runs it), then smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_full
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo rc=$rc $?
