cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.log 2>&1
rc=$?; echo "rc=$rc"; python3 -c "
import json
l=[x for x in open('gpurun_out/bench_final.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'], d['roofline']['traffic'], d.get('traffic_source'))
"
exit $rc
