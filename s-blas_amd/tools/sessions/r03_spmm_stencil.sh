# SpMM (n = 64) with a 27-point stencil A: row forms (fill threshold 0.25, the
# default: the stencil's 16-row blocks fill ~17%, so no MFMA tile) vs the MFMA
# B-panel tile (threshold 0.15), checked against the oracle; kernel trace of the MFMA run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_spmm_stencil
mkdir -p $O
T="timeout -k 10"
B="s-blas_amd/tools/bench_spmm.py --stencil 100 --no-cpu-baseline --steps 10"
for f in 0.25 0.15 0.10; do
  SBLAS_SPMM_MFMA_FILL=$f $T 400 python $B --check > $O/bench_fill$f.json 2> $O/bench_fill$f.err || { tail -20 $O/bench_fill$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_fill$f.json')); print('fill $f', d['kernel_ms_max_over_ranks'], d['value'], d['roofline']['frac'], d.get('check_vs_oracle'))"
done
SBLAS_SPMM_MFMA_FILL=0.15 $T 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $B > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-160 | head -6
echo done
