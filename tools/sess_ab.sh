cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 5 --no-c4 --no-cpu-baseline > gpurun_out/bench_gw.log 2>&1
rc=$?; echo "rc=$rc"; python3 -c "
import json
l=[x for x in open('gpurun_out/bench_gw.log') if x.startswith('{')][-1]
d=json.loads(l); print(json.dumps(d.get('general_wave'))); print(d['value'], d['verified'])
" || tail -20 gpurun_out/bench_gw.log
exit $rc
