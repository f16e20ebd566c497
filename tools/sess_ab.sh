cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
POPORON_AMD_LIB=build/f2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_f2.log 2>&1
rc=$?; echo "tests f2 rc=$rc"; tail -2 gpurun_out/t_f2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/exp_bench.py build/f4.so build/f2.so build/f4.so build/f2.so > gpurun_out/ab_f2.log 2>&1; echo "ab rc=$?"; cut -c1-330 gpurun_out/ab_f2.log
