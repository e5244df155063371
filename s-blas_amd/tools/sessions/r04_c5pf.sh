#!/bin/bash
# round 4: CSR5 tile with phased loads + prefetched row ends (SBLAS_C5_PF=1, default) vs plain (=0)
set -o pipefail
O=gpurun_out/r04_c5pf; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_spmv_gpu.py -k "csr5" \
  "tests/test_configs_gpu.py::test_config2_full_size" tests/test_kernels_gpu.py -k "csr5 or config2" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for PF in 0 1 0 1; do
  SBLAS_C5_PF=$PF timeout -k 10 300 python s-blas_amd/tools/exp_split.py --variants csr5,csr5p8 > $O/split_pf$PF.jsonl 2>>$O/err.log || exit 1
  sed "s/^/pf$PF /" $O/split_pf$PF.jsonl
done
