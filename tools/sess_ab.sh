cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# the fused alternatives of the split decode: traffic and kernel times
for path in single wave; do
  for c in FETCH_SIZE WRITE_SIZE; do
    lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    POPORON_AMD_DECODE_PATH=$path timeout -k 10 200 rocprofv3 --pmc $c -d gpurun_out/fused_$path/roundtrip_$lc -o pmc --output-format csv -- python3 tools/kernel_driver.py --mode roundtrip --reps 3 > gpurun_out/fused_${path}_$lc.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py gpurun_out/fused_$path --json gpurun_out/fused_${path}_traffic.json > gpurun_out/fused_${path}_traffic.txt 2>&1
  cat gpurun_out/fused_${path}_traffic.txt
  POPORON_AMD_DECODE_PATH=$path timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fused_${path}_prof -o run --output-format csv -- python3 tools/kernel_driver.py --mode roundtrip --reps 3 > gpurun_out/fused_${path}_prof.log 2>&1 || exit $?
  find gpurun_out/fused_${path}_prof -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-6 | head -12
done
