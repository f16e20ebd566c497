cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
POPORON_AMD_LIB=build/bm2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bm2.log 2>&1
rc=$?; echo "tests bm2 rc=$rc"; tail -3 gpurun_out/t_bm2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/exp_bench.py build/bm1.so build/bm2.so build/bm1.so build/bm2.so > gpurun_out/ab_bm2.log 2>&1; echo "ab rc=$?"; cut -c1-420 gpurun_out/ab_bm2.log
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 150 rocprofv3 --pmc $grp -d gpurun_out/pmcbs/p$i -o pmc --output-format csv -- python3 tools/probes/bitslice_run.py --sizes 20 --reps 2 > gpurun_out/pmcbs_$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -c 1500 gpurun_out/bench.log
