# r06w: SpTRSV pull with a workgroup-scope store before the agent-scope one (same-XCD consumers see x_i in L2 first), config 5 A/B
set -o pipefail
mkdir -p gpurun_out/r06w
for i in 1 2; do
  timeout -k 10 300 python -u s-blas_amd/tools/exp_trsv.py --reps 5 > gpurun_out/r06w/def_$i.jsonl 2>> gpurun_out/r06w/err.log || exit 1
  SBLAS_LIB=s-blas_amd/alt/libsblas.so timeout -k 10 300 python -u s-blas_amd/tools/exp_trsv.py --reps 5 > gpurun_out/r06w/dual_$i.jsonl 2>> gpurun_out/r06w/err.log || exit 1
done
