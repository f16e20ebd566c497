cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -3 gpurun_out/tests_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; echo "bench rc=$?"
python3 -c "
import json
l=[x for x in open('gpurun_out/bench_full.log') if x.startswith('{')][-1]
d=json.loads(l)
print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'])
g=d['general_params']
print(g['encode_cw_per_s'], g['decode_cw_per_s'], g['encode_ms'], g['decode_ms'], json.dumps(g['decode_kernels_ms']), g['verified'])
"
