# r06e: solo plans as hybrid items (narrow + one wide sub-item per CU): tests, then timings
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_spmv_gpu.py tests/test_configs_gpu.py -k "xsort or solo or empty or auto or config2_full" > gpurun_out/r06e/tests.log 2>&1 && \
timeout -k 10 500 python -u s-blas_amd/tools/exp_opts.py --mats rmat21,synth,stencil27,stencil7 --rounds 2 \
  --opts '[{}, {"det": 1}]' > gpurun_out/r06e/xs.jsonl 2> gpurun_out/r06e/xs.err
