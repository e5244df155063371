#!/bin/bash
# round 4: BASELINE configs[0] (test_spmv f qh768, the reference's results.csv case) through
# the ported CLI: per-call wall clock of the reference operator API (host pointers, device
# memory allocated and freed per call, as in the reference), 1 and 2 GPUs (ordinals wrap)
set -o pipefail
O=gpurun_out/r04_cfg1; mkdir -p $O
for g in 1 2; do
  for k in 1 2; do
    timeout -k 10 120 s-blas_amd/bin/test_spmv f tests/golden/qh768.mtx $g 20 $k f > $O/qh768_g${g}_k$k.txt 2>&1 || { tail $O/qh768_g${g}_k$k.txt; exit 1; }
    grep -i "average\|Average" $O/qh768_g${g}_k$k.txt | head -3 | sed "s/^/g$g k$k: /"
  done
done
# the SpMM row of results.csv: qh768 x 128 dense columns, 1 and 2 GPUs (run_test.py:146-160's argv)
for g in 1 2; do
  timeout -k 10 120 s-blas_amd/bin/test_spmm tests/golden/qh768.mtx 128 $g 1 > $O/spmm_qh768_g$g.txt 2>&1 || { tail $O/spmm_qh768_g$g.txt; exit 1; }
  grep -i "SPMM\|check" $O/spmm_qh768_g$g.txt | head -3 | sed "s/^/spmm g$g: /"
done
