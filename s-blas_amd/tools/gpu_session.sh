#!/bin/bash
# One GPU-box session: parity tests, CLI clones, bench variants, rocprof
# kernel trace and PMC traffic passes.  Every GPU step has its own timeout and
# the chain stops at the first failure.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
STEP="${1:-all}"
run() { echo "[$(date +%T)] $*"; }
if [[ $STEP == all || $STEP == tests ]]; then
  run tests
  timeout -k 10 900 python -m pytest tests/ -q -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [[ $STEP == all || $STEP == cli ]]; then
  run cli
  timeout -k 10 300 ./s-blas_amd/bin/test_spmv f tests/golden/qh768.mtx 1 3 1 f > $O/cli_spmv_1.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_spmv f tests/golden/qh768.mtx 2 3 2 f --ref-loader > $O/cli_spmv_2.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_spmv g 8000 4 2 3 > $O/cli_spmv_g.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_spmm tests/golden/qh768.mtx 128 2 1 > $O/cli_spmm.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_sptrsv -n 1 -rhs 1 -forward -mtx tests/golden/ash85.mtx > $O/cli_sptrsv.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_sptrsv -n 1 -rhs 1 -backward -mtx tests/golden/qh768.mtx -opt 1 > $O/cli_sptrsv_b.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_sptrsv -n 3 -rhs 1 -forward -mtx tests/golden/qh768.mtx > $O/cli_sptrsv_mgpu.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_sptrsv -n 2 -rhs 4 -backward -mtx tests/golden/ash85.mtx > $O/cli_sptrsm.log 2>&1 &&
  timeout -k 10 300 ./s-blas_amd/bin/test_sptrans -n 4 -csr -mtx tests/golden/qh768.mtx > $O/cli_sptrans.log 2>&1 || { echo cli failed; tail -5 $O/cli_*.log; exit 1; }
  tail -n 2 $O/cli_*.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run bench
  for a in panel rowsplit csr5; do for c in random prefix; do
    timeout -k 10 300 python bench.py --algo $a --cols $c --no-cpu-baseline > $O/bench_${a}_${c}.log 2>&1 || exit 1
  done; done
  timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || exit 1
  grep -h '^{' $O/bench_*.log | cut -c1-400
fi
if [[ $STEP == all || $STEP == prof ]]; then
  run prof
  for a in panel rowsplit csr5; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$a -o run --output-format csv -- python bench.py --algo $a --no-cpu-baseline > $O/prof_$a.log 2>&1 || exit 1
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$a -o run --output-format csv -- python bench.py --algo $a --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc_fetch_$a.log 2>&1 || exit 1
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$a -o run --output-format csv -- python bench.py --algo $a --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc_write_$a.log 2>&1 || exit 1
    timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pmc_l2_$a -o run --output-format csv -- python bench.py --algo $a --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc_l2_$a.log 2>&1 || exit 1
  done
  for a in panel rowsplit csr5; do
    case $a in panel) k=k_spmv_panel,k_panel_reduce;; rowsplit) k=k_spmv_rowsplit;; csr5) k=k_spmv_csr5,k_csr5_calibrate;; esac
    python3 s-blas_amd/tools/pmc_traffic.py --kernel $k --fetch $O/pmc_fetch_$a --write $O/pmc_write_$a --l2 $O/pmc_l2_$a --algorithmic 533000004 --out $O/pmc_$a.json > /dev/null || exit 1
  done
  ls $O/pmc_*.json
fi
if [[ $STEP == prof2 ]]; then
  # kernel-trace summaries of the non-SpMV rows (SpTRSV/SpTRSM, SpMM, transpose, out-of-core)
  run prof2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trsv -o run --output-format csv -- python s-blas_amd/tools/bench_sptrsv.py --rhs 8 --no-cpu-baseline --steps 3 > $O/prof_trsv.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_spmm -o run --output-format csv -- python s-blas_amd/tools/bench_spmm.py > $O/prof_spmm.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tr -o run --output-format csv -- python s-blas_amd/tools/bench_transpose.py --mgpu 2 > $O/prof_tr.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ooc -o run --output-format csv -- python s-blas_amd/tools/bench_ooc.py --reps 1 --chunks 16777216 --streams 2 > $O/prof_ooc.log 2>&1 || exit 1
  ls $O/prof_trsv $O/prof_spmm $O/prof_tr $O/prof_ooc
fi
echo "[$(date +%T)] session done"
