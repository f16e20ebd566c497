cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in oddA oddB; do
  POPORON_AMD_LIB=build/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -3 gpurun_out/t_$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 600 python tools/exp_bench.py build/base.so build/oddA.so build/oddB.so build/base.so build/oddA.so build/oddB.so > gpurun_out/ab_chien.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_chien.log
