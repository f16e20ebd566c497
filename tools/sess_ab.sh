cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in bp_px4 bp_px5 bp_px6; do
  POPORON_AMD_LIB=$PWD/build/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q -k "era or erasure" --timeout 120 --timeout-method thread > gpurun_out/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -2 gpurun_out/tests_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for r in 1 2; do
  timeout -k 10 600 python tools/exp_bench.py build/bp_base.so build/bp_px4.so build/bp_px5.so build/bp_px6.so > gpurun_out/bp_ab_$r.log 2>&1 || exit $?
  cat gpurun_out/bp_ab_$r.log
done
