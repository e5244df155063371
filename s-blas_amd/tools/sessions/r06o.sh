# r06o: xsort LDS rows 16384 (default) vs 19456 (alt build), paired vs solo narrow items, config 2 / stencil27 / R-MAT
set -o pipefail
mkdir -p gpurun_out/r06o
for i in 1 2; do
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --no-check --reps 10 --opts '[{}, {"xs_solo": 1}]' > gpurun_out/r06o/def_$i.jsonl 2>> gpurun_out/r06o/err.log || exit 1
  SBLAS_LIB=s-blas_amd/alt/libsblas.so timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --reps 10 --opts '[{}, {"xs_solo": 1}]' > gpurun_out/r06o/alt_$i.jsonl 2>> gpurun_out/r06o/err.log || exit 1
done
