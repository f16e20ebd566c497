#!/bin/bash
# Forney kernel with and without its apply (POPORON_AMD_STOP_AT=5), kernel times from the bench's HIP events
cd "${GRAFT_REPO_ROOT:-.}"
for st in 0 5; do
  POPORON_AMD_STOP_AT=$st timeout -k 10 200 python -u bench.py --no-c4 --no-cpu-baseline --no-host --no-latency --no-erasure > gpurun_out/abl_$st.log 2>&1
  python3 -c "
import json; l=[x for x in open('gpurun_out/abl_$st.log') if x.startswith('{')][-1]; d=json.loads(l)
print('stop_at=$st', d['ms_per_step'], {k: v['ms_per_step'] for k,v in d['kernels'].items()})"
done
