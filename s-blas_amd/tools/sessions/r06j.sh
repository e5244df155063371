# r06j: xsort entry-stream touches through the scalar cache (experiment builds), A/B
set -o pipefail
mkdir -p gpurun_out/r06j
for i in 1 2; do
  for v in prev pf1 pf2 pf2a16 pf1a16; do
    SBLAS_LIB=s-blas_amd/alt_$v/libsblas.so timeout -k 10 200 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --opts '[{}]' --reps 8 > gpurun_out/r06j/${v}_$i.jsonl 2>> gpurun_out/r06j/err.log || exit 1
  done
  timeout -k 10 200 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --opts '[{}]' --reps 8 > gpurun_out/r06j/pf0_$i.jsonl 2>> gpurun_out/r06j/err.log || exit 1
done
