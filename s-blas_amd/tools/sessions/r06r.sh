# r06r: xsort stress -- 2000 launches per handle on config 2 and R-MAT 21, every y against the oracle bound, deterministic handles bitwise equal
set -o pipefail
mkdir -p gpurun_out/r06r
timeout -k 10 400 python -u s-blas_amd/tools/stress_xsort.py --launches 2000 --matrix synth > gpurun_out/r06r/stress_synth.json 2> gpurun_out/r06r/err.log || exit 1
timeout -k 10 400 python -u s-blas_amd/tools/stress_xsort.py --launches 2000 --matrix rmat21 > gpurun_out/r06r/stress_rmat21.json 2>> gpurun_out/r06r/err.log || exit 1
