cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_generic_wave.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_gw.log 2>&1 && \
timeout -k 10 400 python -u tools/general_lat.py > gpurun_out/general_lat_auto.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/tests_gw.log
exit $rc
