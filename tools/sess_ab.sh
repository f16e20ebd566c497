cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; echo "bench rc=$?"
python3 -c "
import json
l=[x for x in open('gpurun_out/bench_full.log') if x.startswith('{')][-1]
d=json.loads(l)
print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'])
print(json.dumps({k: d[k] for k in ('erasure_decode_32', 'errata_decode_16e8') if k in d})[:800])
g=d['general_params']
print(json.dumps(g))
"
