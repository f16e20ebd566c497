cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/tests_all.log
exit $rc
