# r06k: xsort group-split narrow ranges (solo plans): parity (small + full-size R-MAT), then A/B timing
set -o pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_spmv_gpu.py -k "xsort or rmat or auto" -m gpu > gpurun_out/r06k/pytest_small.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_configs_gpu.py -k rmat21 -m gpu > gpurun_out/r06k/pytest_rmat21.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats rmat21 --no-check --reps 10 --opts '[{}, {"xs_gsplit": 2}, {"xs_gsplit": 4}]' > gpurun_out/r06k/rmat_$i.jsonl 2>> gpurun_out/r06k/err.log || exit 1
  SBLAS_LIB=s-blas_amd/alt_head/libsblas.so timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats rmat21,synth,stencil27 --no-check --reps 10 --opts '[{}]' > gpurun_out/r06k/head_$i.jsonl 2>> gpurun_out/r06k/err.log || exit 1
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27 --no-check --reps 10 --opts '[{}]' > gpurun_out/r06k/new_$i.jsonl 2>> gpurun_out/r06k/err.log || exit 1
done
