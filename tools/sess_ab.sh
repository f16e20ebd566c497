cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -k "overlap" --timeout 120 --timeout-method thread > gpurun_out/tests_ov.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/tests_ov.log
if [ $rc -ne 0 ]; then exit $rc; fi
Q="--no-c4 --no-erasure --no-mixed --no-host --no-latency --no-general --no-cpu-baseline --steps 20"
for r in 1 2 3; do
  for ov in 0 1 2; do
    timeout -k 10 300 python bench.py $Q --overlap $ov > gpurun_out/ov_${ov}_$r.log 2>&1 || exit $?
    python3 -c "
import json
l=[x for x in open('gpurun_out/ov_${ov}_$r.log') if x.startswith('{')][-1]
d=json.loads(l)
print('overlap=$ov rep=$r', d['value'], d['ms_per_step'], d['verified'])
"
  done
done
