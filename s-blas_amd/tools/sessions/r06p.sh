# r06p: xsort with the wide ranges' reduce fused into the kernel (test hook xs_fuse): parity, then A/B
set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_spmv_gpu.py -k "xsort or auto" -m gpu > gpurun_out/r06p/pytest_small.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py -k "xsort or rmat21 or deterministic" -m gpu > gpurun_out/r06p/pytest_cfg.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u s-blas_amd/tools/exp_opts.py --mats synth,stencil27,rmat21 --no-check --reps 10 --opts '[{}, {"xs_fuse": 1}, {"det": 1}, {"det": 1, "xs_fuse": 1}]' > gpurun_out/r06p/ab_$i.jsonl 2>> gpurun_out/r06p/err.log || exit 1
done
