cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic_wave.py -x -v --timeout 120 --timeout-method thread -k large > gpurun_out/tests_gw.log 2>&1
rc=$?; echo "rc=$rc"; tail -8 gpurun_out/tests_gw.log
exit $rc
