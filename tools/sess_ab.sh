cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_nrsplit.py tests/test_gpu_parity.py tests/test_gpu_single.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_nr.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/tests_nr.log | tail -15
