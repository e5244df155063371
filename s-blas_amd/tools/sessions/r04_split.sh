#!/bin/bash
# round 4: config 2's heavy / light rows per kernel, CSR5 column panels on heavy rows only
set -o pipefail
O=gpurun_out/r04_split; mkdir -p $O
timeout -k 10 500 python s-blas_amd/tools/exp_split.py > $O/split.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
cat $O/split.jsonl
