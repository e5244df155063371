# round 3: counters of the tall-tile SpMM kernel (config 4), one rocprofv3 pass per counter group
set -o pipefail
export TMPDIR=/tmp
bash s-blas_amd/tools/prof_counters_cmd.sh k_spmm_ttile gpurun_out/r03_spmm_pmc s-blas_amd/tools/bench_spmm.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r03_spmm_pmc.log 2>&1
echo rc=$?
tail -3 gpurun_out/r03_spmm_pmc.log
