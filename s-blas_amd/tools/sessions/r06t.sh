# r06t: every SpMV kernel on the structured stand-ins (is AUTO's xsort the best pick on each?)
set -o pipefail
mkdir -p gpurun_out/r06t
for algo in 1 2 4 5; do
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats rmat21,stencil27,stencil7 --algo $algo --reps 10 --opts '[{}]' >> gpurun_out/r06t/algos.jsonl 2>> gpurun_out/r06t/err.log || exit 1
done
