# r06g: row split with non-temporal y / partial stores (A/B against alt_prev, SBLAS_LIB), P = 4 and 8
set -o pipefail
mkdir -p gpurun_out/r06g
for i in 1 2; do
  SBLAS_LIB=s-blas_amd/alt_prev/libsblas.so timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth --algo 1 --opts '[{}, {"panels": 8, "rs_panel": 1}]' > gpurun_out/r06g/prev_$i.jsonl 2>> gpurun_out/r06g/err.log || exit 1
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth --algo 1 --opts '[{}, {"panels": 8, "rs_panel": 1}]' > gpurun_out/r06g/new_$i.jsonl 2>> gpurun_out/r06g/err.log || exit 1
done
