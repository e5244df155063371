# round 3: CSR5 over XCD column panels -- parity, config-2 bench (panel vs plain), N = 8 slices, kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_csr5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_spmv_gpu.py -k "csr5" "tests/test_configs_gpu.py::test_config2_full_size" "tests/test_configs_gpu.py::test_config2_alpha_beta_zero" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --algo csr5 --no-cpu-baseline --no-rowsplit-beside > $O/bench_csr5_panel.json 2> $O/b1.err &&
SBLAS_CSR5_PANEL=0 timeout -k 10 300 python bench.py --algo csr5 --no-cpu-baseline --no-rowsplit-beside > $O/bench_csr5_plain.json 2> $O/b2.err &&
SBLAS_PANELS=8 timeout -k 10 300 python bench.py --algo csr5 --no-cpu-baseline --no-rowsplit-beside > $O/bench_csr5_panel8.json 2> $O/b3.err &&
SBLAS_PANELS=2 timeout -k 10 300 python bench.py --algo csr5 --no-cpu-baseline --no-rowsplit-beside > $O/bench_csr5_panel2.json 2> $O/b4.err &&
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos csr5,panel,xsort > $O/slice_panel.jsonl 2> $O/s1.err &&
SBLAS_CSR5_PANEL=0 timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 8 --algos csr5 > $O/slice_plain.jsonl 2> $O/s2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --algo csr5 --no-cpu-baseline --no-rowsplit-beside > $O/bench_csr5_prof.json 2> $O/prof.err
echo rc=$?
for f in $O/bench_*.json; do echo $f; grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], d['roofline']['frac'])"; done
cat $O/slice_*.jsonl
