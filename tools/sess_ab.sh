cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
python3 -c "
import json
l=[x for x in open('gpurun_out/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'])
print(json.dumps(d.get('general_params')))
print(json.dumps(d['roofline']['kernels_ms']))
"
