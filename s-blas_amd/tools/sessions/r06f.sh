# r06f: A/B of the xsort epilogue/hybrid-solo build against the previous xsort (alt_prev, SBLAS_LIB)
set -o pipefail
mkdir -p gpurun_out/r06f
for i in 1 2; do
  SBLAS_LIB=s-blas_amd/alt_prev/libsblas.so timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats rmat21,synth,stencil27,stencil7 --no-check --opts '[{}]' > gpurun_out/r06f/prev_$i.jsonl 2>> gpurun_out/r06f/err.log || exit 1
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats rmat21,synth,stencil27,stencil7 --no-check --opts '[{}]' > gpurun_out/r06f/new_$i.jsonl 2>> gpurun_out/r06f/err.log || exit 1
done
