cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/tests_all.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/nr_single.py > gpurun_out/nr_single.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/nr_single.log
