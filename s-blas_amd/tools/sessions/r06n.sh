# r06n: SpTRSV XCD-blocked pull (workgroup-scope publication inside an XCD's block) vs the pull executor, config 5
set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 400 python -u s-blas_amd/tools/exp_trsv.py --rounds 2 --reps 5 --opts '[{}, {"trsv_xcd": 1}]' > gpurun_out/r06n/trsv.jsonl 2> gpurun_out/r06n/err.log || exit 1
timeout -k 10 400 python -u s-blas_amd/tools/exp_trsv.py --algo 3 --rounds 2 --reps 5 --opts '[{}, {"trsv_xcd": 1}, {"trsv_xcd": 1, "trsv_xcd_waves": 4}, {"trsv_xcd": 1, "trsv_xcd_waves": 2}]' > gpurun_out/r06n/trsv_lvl.jsonl 2>> gpurun_out/r06n/err.log || exit 1
