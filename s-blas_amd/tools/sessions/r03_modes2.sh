# round 3: x gathers -- L2-resident gathers (mode 16) vs product, and the unpaired 16384-row items
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_modes2
mkdir -p $O
rc=0
for v in "SBLAS_XS_MODE=16" "SBLAS_XS_PAIR=0" "SBLAS_XS_MODE=0"; do
  env $v timeout -k 10 240 python3 s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort > $O/$v.jsonl 2> $O/$v.err || { rc=$?; break; }
  echo "$v"; cat $O/$v.jsonl
done
echo rc=$rc
