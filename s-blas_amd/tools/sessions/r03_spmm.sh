# round 3: tall-tile SpMM -- parity first, then the config-4 bench (tall tile vs C tile) under rocprofv3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_spmm
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "tests/test_kernels_gpu.py::test_spmm" "tests/test_kernels_gpu.py::test_spmm_two_handles_two_streams" "tests/test_configs_gpu.py::test_config4_spmm_full_size" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SBLAS_SPMM_TTILE=1 SBLAS_SPMM_TTSTAT=1 timeout -k 10 300 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > $O/bench_tt.json 2> $O/bench_tt.err &&
SBLAS_SPMM_TTILE=1 SBLAS_SPMM_TTSTAT=1 SBLAS_SPMM_TTWIN=1 timeout -k 10 300 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > $O/bench_tt_win1.json 2> $O/bench_tt_win1.err &&
timeout -k 10 300 python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > $O/bench_ct.json 2> $O/bench_ct.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python s-blas_amd/tools/bench_spmm.py --no-cpu-baseline > $O/bench_tt_prof.json 2> $O/prof.err
echo rc=$?
grep -h "tt plan" $O/*.err
for f in $O/bench_*.json; do echo $f; grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['kernel_ms_max_over_ranks'], d['plan_build_s_rank0'])"; done
