cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ext_batchlat.py > gpurun_out/ext_batchlat.log 2>&1 && \
timeout -k 10 300 python -u tools/ext_batchlat.py --params 8,0x11D,1,1,16 >> gpurun_out/ext_batchlat.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/ext_batchlat.log | tail -12
exit $rc
