#!/bin/bash
# round 4: counters of the CSR5 kernel on config 2's light rows vs its heavy rows
set -o pipefail
O=gpurun_out/r04_c5pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in light heavy; do
  bash s-blas_amd/tools/prof_counters_cmd.sh k_spmv_csr5 $O/$P s-blas_amd/tools/exp_split.py --parts $P --variants csr5 --reps 3 || exit 1
done
python3 -c "
import json
for p in ('light','heavy'):
    d=json.load(open('$O/'+p+'/summary.json')); print(p, json.dumps(d)[:1500])
"
