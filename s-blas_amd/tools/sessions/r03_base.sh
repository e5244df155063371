set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_base
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/prof.err
echo rc=$?
