#!/bin/bash
# device CSR5 plan + SpTRSM push lane mappings: targeted tests, then plan-build timing
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "csr5 or sptrsm or sptrsv_reference" > gpurun_out/t_c5trsm.log 2>&1 || { tail -30 gpurun_out/t_c5trsm.log; exit 1; }
tail -1 gpurun_out/t_c5trsm.log
for hp in 0 1; do
  SBLAS_CSR5_HOSTPLAN=$hp $T 300 python bench.py --algo csr5 --steps 5 --warmup 2 --no-cpu-baseline --no-rowsplit-beside > gpurun_out/b_c5_$hp.json 2> gpurun_out/b_c5_$hp.err || { tail -5 gpurun_out/b_c5_$hp.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b_c5_$hp.json')); print('hostplan=$hp', d['plan'], d['kernel_ms'])"
done
$T 400 python s-blas_amd/tools/bench_sptrsv.py --steps 3 --rhs 4,16 --no-cpu-baseline > gpurun_out/bst_rhs.json 2> gpurun_out/bst_rhs.err || { tail -5 gpurun_out/bst_rhs.err; exit 1; }
cat gpurun_out/bst_rhs.json
$T 300 python s-blas_amd/tools/bench_slice.py --worlds 8,4 --algos xsort,panel,rowsplit,csr5 --floor > gpurun_out/slice.jsonl 2> gpurun_out/slice.err || { tail -5 gpurun_out/slice.err; exit 1; }
cat gpurun_out/slice.jsonl
for v in "SBLAS_XS_FUSE=1" "SBLAS_XS_K24=2" "SBLAS_XS_ALLWIDE=1"; do
  echo "$v"; env $v $T 200 python s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort > gpurun_out/slice_v.jsonl 2>&1 || { tail -5 gpurun_out/slice_v.jsonl; exit 1; }
  cat gpurun_out/slice_v.jsonl
done
