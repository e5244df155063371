#!/bin/bash
# round 4: CSR5 on the 27-/7-point stencils, commit e09f70e's tree (_old_e09, built
# from that commit) against HEAD, alternated: where did 0.70 -> 0.62 come from?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_stencilreg; mkdir -p $O
B="--algo csr5 --no-cpu-baseline --no-rowsplit-beside --no-config3"
for v in old1 new1 old2 new2; do
  case $v in old*) D=_old_e09;; *) D=.;; esac
  for mtx in stencil27 stencil7; do
    (cd $D && timeout -k 10 300 python bench.py --matrix $mtx $B) > $O/bench_${mtx}_$v.json 2>>$O/err.log || exit 1
  done
  python3 -c "
import json
print('$v', [(m,)+tuple((lambda d:(d['ms_per_step'],d['roofline']['frac']))(json.loads(open('$O/bench_'+m+'_$v.json').read().strip().splitlines()[-1]))) for m in ('stencil27','stencil7')])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run --output-format csv -- python3 bench.py --matrix stencil27 $B > /dev/null 2>>$O/err.log || exit 1
cd _old_e09 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../$O/prof_old -o run --output-format csv -- python3 bench.py --matrix stencil27 $B > /dev/null 2>>../$O/err.log || exit 1
cd .. && for v in new old; do python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
    if 'sblas' in r['Name']: print('$v', r['Name'].split('(')[0][-50:], r['Calls'], r['AverageNs'])"; done
