# round 3: xsort epilogue with non-temporal y / partial stores (SBLAS_XS_NTSTORE) vs plain, A/B/A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_ntstore
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-rowsplit-beside > $O/bench_plain_$i.json 2>> $O/e.err || exit 1
  SBLAS_XS_NTSTORE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-rowsplit-beside > $O/bench_nt_$i.json 2>> $O/e.err || exit 1
done
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --algos xsort > $O/slice_plain.jsonl 2>> $O/e.err &&
SBLAS_XS_NTSTORE=1 timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --algos xsort > $O/slice_nt.jsonl 2>> $O/e.err
echo rc=$?
for f in $O/bench_*.json; do echo $f $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'], d['warm']['ms_per_step'])"); done
cat $O/slice_*.jsonl
