# heavy-range partials stored sc1 (write-through, not left dirty in L2 at the
# kernel boundary; SBLAS_XS_SC1PART=1) vs plain stores, separate reduce launch
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_sc1part
mkdir -p $O
T="timeout -k 10"
B="bench.py --no-cpu-baseline --no-rowsplit-beside"
for i in 1 2 3; do
  $T 300 python $B > $O/bench_base_$i.json 2> $O/bench_base_$i.err || { tail -20 $O/bench_base_$i.err; exit 1; }
  SBLAS_XS_SC1PART=1 $T 300 python $B > $O/bench_sc1_$i.json 2> $O/bench_sc1_$i.err || { tail -20 $O/bench_sc1_$i.err; exit 1; }
done
for f in $O/bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['kernel_ms'], d['roofline']['frac'], d['warm']['kernel_ms'])"; done
S="s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort"
SBLAS_XS_SC1PART=0 $T 300 python $S > $O/slice_base.jsonl 2> $O/slice_base.err || { tail -20 $O/slice_base.err; exit 1; }
SBLAS_XS_SC1PART=1 $T 300 python $S > $O/slice_sc1.jsonl 2> $O/slice_sc1.err || { tail -20 $O/slice_sc1.err; exit 1; }
cat $O/slice_base.jsonl $O/slice_sc1.jsonl
echo done
