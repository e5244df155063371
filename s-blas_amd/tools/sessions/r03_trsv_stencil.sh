# SpTRSV on the lower triangle of 3-D stencils (FEM kind): every executor
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_trsv_stencil
mkdir -p $O
T="timeout -k 10"
for g in 64 100; do
  for pts in 27 7; do
    $T 300 python s-blas_amd/tools/bench_sptrsv.py --stencil $g --points $pts --steps 3 --no-cpu-baseline > $O/trsv_s${pts}_g$g.json 2> $O/trsv_s${pts}_g$g.err || { tail -20 $O/trsv_s${pts}_g$g.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/trsv_s${pts}_g$g.json'))
print('$pts-pt g=$g n', d['config']['n'], 'levels', d['config']['levels'], {k: (v['ms'], '%.1e' % v['rel_l1_vs_xref']) for k, v in d['executors'].items()})"
  done
done
echo done
