# r06d: (1) R-MAT solo plans, narrow items re-cut at 1/K of the cap
# (xs_nsplit K); (2) row split / CSR5 on config 2 over 4 vs 8 vs 2 XCD panels
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 400 python -u s-blas_amd/tools/exp_opts.py --mats rmat21 --rounds 2 \
  --opts '[{"xs_nsplit": 1}, {"xs_nsplit": 2}, {"xs_nsplit": 3}, {"xs_nsplit": 4}, {"xs_nsplit": 6}]' \
  > gpurun_out/r06d/rmat.jsonl 2> gpurun_out/r06d/rmat.err && \
timeout -k 10 400 python -u s-blas_amd/tools/exp_opts.py --mats synth --algo 1 --rounds 2 \
  --opts '[{}, {"panels": 8, "rs_panel": 1}, {"panels": 2, "rs_panel": 1}]' \
  > gpurun_out/r06d/rs.jsonl 2> gpurun_out/r06d/rs.err && \
timeout -k 10 400 python -u s-blas_amd/tools/exp_opts.py --mats synth --algo 2 --rounds 2 \
  --opts '[{}, {"panels": 8, "csr5_panel": 1}, {"panels": 2, "csr5_panel": 1}]' \
  > gpurun_out/r06d/c5.jsonl 2> gpurun_out/r06d/c5.err
