#!/bin/bash
# the cyclic exchange (plain and two-half overlapped) through RCCL on one GPU:
# torchrun with one rank, --dist-always, SBLAS_DIST_XCHG_W1=1 (all-gathers and
# placements run although the world is one rank), checked against the oracle
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export HSA_ENABLE_IPC_MODE_LEGACY=0 SBLAS_DIST_XCHG_W1=1
i=0
for extra in "" "--overlap" "--overlap --algo panel"; do
  i=$((i+1))
  $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29700+i)) \
     bench.py --gpus 1 --steps 10 --warmup 3 --dist-always --check --no-cpu-baseline $extra > gpurun_out/nccl2_$i.json 2> gpurun_out/nccl2_$i.err || { tail -20 gpurun_out/nccl2_$i.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/nccl2_$i.json') if l.startswith('{')][-1])
print('$extra', 'check', d.get('check_vs_oracle'), 'value', d['value'], 'ms', d['ms_per_step'], 'exch', d.get('exchange_ms_max_over_ranks'), d['config'].get('partition'))
"
done
