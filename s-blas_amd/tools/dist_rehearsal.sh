#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: several ranks share the
# GPU and talk over gloo (RCCL refuses two ranks on one GPU).  Each run checks
# the assembled y against the oracle (--check).  Outputs under gpurun_out/.
set -o pipefail
O=gpurun_out; mkdir -p $O
port=29611
# (exchange, partition, algorithms): cyclic row chunks are the allgather default
for np in 2 3 4; do for combo in "allgather cyclic xsort panel rowsplit csr5" "allgather nnz xsort panel" \
    "allreduce nnz panel csr5"; do
  set -- $combo; ex=$1; part=$2; shift 2
  for algo in "$@"; do
  port=$((port+1))
  L=$O/rehearsal_${np}_${ex}_${part}_${algo}.log
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $np --dist-backend gloo \
    --nrows 200000 --steps 3 --warmup 1 --check --exchange $ex --partition $part --algo $algo \
    > $L 2>&1 || { echo "FAIL np=$np $ex $part $algo"; tail -20 $L; exit 1; }
  grep -h '^{' $L | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); c=d.get('check_vs_oracle'); print('np=$np $ex $part $algo check=', c, d['value']); sys.exit(0 if c else 1)" || exit 1
done; done; done
# torchrun with one rank over RCCL (the driver's N=1 launch shape)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port $((port+1)) bench.py --gpus 1 --no-cpu-baseline --check --nrows 200000 > $O/rehearsal_1_nccl.log 2>&1 || exit 1
grep -h '^{' $O/rehearsal_1_nccl.log | cut -c1-200
# SpMM (G2): rows of A by nnz, B replicated, C slices all-gathered
for np in 2 3; do
  port=$((port+7))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $port s-blas_amd/tools/bench_spmm.py --dist-backend gloo \
    --mrows 1000 --kcols 100000 --nnz 500000 --steps 3 --warmup 1 > $O/rehearsal_spmm_${np}.log 2>&1 || { echo "FAIL spmm np=$np"; tail -20 $O/rehearsal_spmm_${np}.log; exit 1; }
  grep -h '^{' $O/rehearsal_spmm_${np}.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); e=d['max_rel_err_32_rows']; print('spmm np=$np err=', e); sys.exit(0 if e < 1e-12 else 1)" || exit 1
done
