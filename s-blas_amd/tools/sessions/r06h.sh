# r06h: deterministic xsort with the next claim's gathers issued before the turn wait (A/B vs alt_prev)
set -o pipefail
mkdir -p gpurun_out/r06h
for i in 1 2; do
  SBLAS_LIB=s-blas_amd/alt_prev/libsblas.so timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --opts '[{"det": 1}]' > gpurun_out/r06h/prev_$i.jsonl 2>> gpurun_out/r06h/err.log || exit 1
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --opts '[{"det": 1}, {}]' > gpurun_out/r06h/new_$i.jsonl 2>> gpurun_out/r06h/err.log || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_configs_gpu.py tests/test_spmv_gpu.py -k "deterministic or det" > gpurun_out/r06h/tests.log 2>&1
