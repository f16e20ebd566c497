cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_generic_wave.py tests/test_gpu_parity.py tests/test_gpu_nrsplit.py tests/test_gpu_single.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_gw.log 2>&1 && \
timeout -k 10 300 python -u tools/gw_phases.py > gpurun_out/gw_phases.log 2>&1
rc=$?; echo "rc=$rc"; tail -4 gpurun_out/tests_gw.log; grep -v "^{" gpurun_out/gw_phases.log
exit $rc
