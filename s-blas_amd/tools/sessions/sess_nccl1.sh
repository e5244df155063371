#!/bin/bash
# the N > 1 bench path (RCCL process group, exchange, cold timing) on one GPU:
# torchrun with one rank and --dist-always, every run checked against the oracle
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for extra in "" "--overlap" "--algo csr5 --partition nnz --exchange allreduce" "--algo panel --partition nnz"; do
  i=$((i+1))
  $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600+i)) \
     bench.py --gpus 1 --steps 10 --warmup 3 --dist-always --check --no-cpu-baseline $extra > gpurun_out/nccl1_$i.json 2> gpurun_out/nccl1_$i.err || { tail -20 gpurun_out/nccl1_$i.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/nccl1_$i.json') if l.startswith('{')][-1])
print('$extra', 'check', d.get('check_vs_oracle'), 'value', d['value'], 'ms', d['ms_per_step'], 'exch', d.get('exchange_ms_max_over_ranks'), d['config'].get('algo'), d['config'].get('exchange'))
"
done
