# r06q: fused wide-range reduce on the N > 1 rank slices of config 2 (all-wide / mixed plans)
set -o pipefail
mkdir -p gpurun_out/r06q
for i in 1 2; do
  timeout -k 10 400 python -u s-blas_amd/tools/exp_opts.py --mats slice8,slice4,slice2 --reps 10 --opts '[{}, {"xs_fuse": 1}]' > gpurun_out/r06q/slices_$i.jsonl 2>> gpurun_out/r06q/err.log || exit 1
done
