cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nrsplit.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_nr.log 2>&1
rc=$?; echo "nrsplit tests rc=$rc"; tail -4 gpurun_out/tests_nr.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -3 gpurun_out/tests_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/nr_batchlat.py > gpurun_out/nr_batchlat.log 2>&1 || exit $?
tail -1 gpurun_out/nr_batchlat.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; echo "bench rc=$?"
python3 -c "
import json
l=[x for x in open('gpurun_out/bench_full.log') if x.startswith('{')][-1]
d=json.loads(l)
print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'])
print(json.dumps(d.get('general_params')))
"
