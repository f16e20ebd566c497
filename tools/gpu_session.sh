#!/bin/bash
# tools/gpu_session.sh STEP... -- run GPU steps on the gpurun box, each under
# its own time limit, stopping at the first fault/abort/timeout (exit codes
# other than 0 = ok and 1 = test/assert failure).  Logs go to gpurun_out/.
#   steps: smoke | tests | bench | prof | pmc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { # name limit cmd...
    local name=$1 lim=$2
    shift 2
    echo "== $name: $*" | tee -a gpurun_out/session.log
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping: $name exited $rc" | tee -a gpurun_out/session.log
        exit $rc
    fi
    return 0
}
for step in "$@"; do
    case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests_all) run tests_all 900 python -m pytest tests -m gpu -q ;;
    bench) run bench 600 python bench.py ;;
    beside) # the cross-handle batch / single-call test on each build in build/*.so, then the tree's
        for so in build/*.so; do
            POPORON_AMD_LIB=$so run "beside_$(basename $so .so)" 300 python -u -m pytest tests/test_gpu_fullsize.py \
                -k beside -v -s --timeout 250 --timeout-method thread
        done
        run beside_tree 300 python -u -m pytest tests/test_gpu_fullsize.py -k beside -v -s --timeout 250 \
            --timeout-method thread ;;
    lat) run lat 200 python tools/lat_single.py 2000
         POPORON_AMD_SERVE=0 run lat_noserve 200 python tools/lat_single.py 2000 ;;
    bsz) run bsz 700 bash tools/batch_sizes.sh ;;
    batchwave) POPORON_AMD_DECODE_PATH=wave run batchlat_wave 300 python tools/batch_latency.py ;;
    batchlat) run batchlat 300 python tools/batch_latency.py
              POPORON_AMD_DECODE_PATH=split run batchlat_split 300 python tools/batch_latency.py
              POPORON_AMD_DECODE_PATH=wave run batchlat_wave 300 python tools/batch_latency.py ;;
    latab) # single-call latency of each build/*.so, alternated twice (same box)
        for pass in 1 2; do
            for so in build/*.so; do
                POPORON_AMD_LIB=$so run "latab_$(basename $so .so)_$pass" 200 python tools/lat_single.py 2000
            done
        done ;;
    srvbatch) # batch calls right after a single call, each build in build/*.so (+ the server off)
        for so in build/*.so; do
            POPORON_AMD_LIB=$so run "srvbatch_$(basename $so .so)" 200 python tools/server_batch.py
        done
        POPORON_AMD_SERVE=0 run srvbatch_noserve 200 python tools/server_batch.py ;;
    ab) # A/B of the experiment builds in build/*.so, alternated twice (same box)
        run ab 900 python tools/exp_bench.py $(ls build/*.so) $(ls build/*.so) ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-host --no-c4 --no-latency --no-mixed --no-general --steps 10 ;;
    gwtests) run gw_tests 400 python -u -m pytest tests/test_gpu_generic_wave.py -x -q --timeout 120 --timeout-method thread ;;
    glat) run glat_wave 300 python tools/general_lat.py --calls 30 --path wave
          run glat_lane 300 python tools/general_lat.py --calls 30 --path lane ;;
    glatauto) run glat_auto 300 python tools/general_lat.py --calls 30 ;;
    gparity) run gparity 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
                 -k "general or generic or short or lfsr" ;;
    gbig) run gbig 400 python -u -m pytest tests/test_gpu_generic_wave.py -x -q --timeout 120 --timeout-method thread \
                 -k "large_batch" ;;
    gwbatch) # general-parameter batch decodes: both families, then PMC of the wave family on RS(255,155)
        for prm in 8,0x11d,1,1,100 4,0x13,1,2,8 6,0x43,1,1,10 7,0x89,1,1,20; do
            for fam in wave lane; do
                POPORON_AMD_GENERIC=$fam run gwb_${fam}_${prm//,/_} 120 python tools/gw_batch.py --params $prm
            done
        done
        POPORON_AMD_GENERIC=wave run gwb_pmc 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
            SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/gwb_pmc \
            -o pmc --output-format csv -- python3 tools/gw_batch.py --params 8,0x11d,1,1,100 --reps 3 ;;
    gwconf) # LDS bank conflicts of the general wave decode (RS(255,155)), then of RS(15,7)
        for prm in 8,0x11d,1,1,100 4,0x13,1,2,8; do
            POPORON_AMD_GENERIC=wave run gwconf_${prm//,/_} 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
                SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
                -d gpurun_out/gwconf_${prm//,/_} -o pmc --output-format csv -- python3 tools/gw_batch.py --params $prm --reps 3
        done ;;
    gwab) # general batch decodes on each build in build/*.so (RS(255,155), RS(127,107), RS(15,7)), alternated twice
        for pass in 1 2; do
            for so in build/gw[A-Z]*.so; do
                for prm in 8,0x11d,1,1,100 7,0x89,1,1,20 4,0x13,1,2,8; do
                    POPORON_AMD_LIB=$so POPORON_AMD_GENERIC=wave run gwab_$(basename $so .so)_${prm//,/_}_$pass 120 \
                        python tools/gw_batch.py --params $prm
                done
            done
        done
        grep -h "M cw/s" gpurun_out/gwab_*.log > gpurun_out/gwab_summary.txt 2>/dev/null
        for f in gpurun_out/gwab_*.log; do echo "$f: $(grep -h 'M cw/s' $f)"; done > gpurun_out/gwab_summary.txt ;;
    gwphase) # general batch decode time up to each phase (build/gwp*.so: GW_PHASE_STOP builds), RS(255,155) and RS(15,7)
        for so in build/gwp*.so; do
            for prm in 8,0x11d,1,1,100 4,0x13,1,2,8; do
                POPORON_AMD_LIB=$so POPORON_AMD_GENERIC=wave run gwp_$(basename $so .so)_${prm//,/_} 120 \
                    python tools/gw_batch.py --params $prm --no-check
            done
        done
        for f in gpurun_out/gwp_*.log; do echo "$f: $(grep -h 'M cw/s' $f)"; done > gpurun_out/gwphase_summary.txt ;;
    pmcab) # the first two SQ counter groups on each build in build/*.so (decode16 round trip)
        for so in build/*.so; do
            b=$(basename $so .so)
            i=0
            for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                       "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY" \
                       "SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
                POPORON_AMD_LIB=$so run pmcab_${b}_$i 300 rocprofv3 --pmc $grp -d gpurun_out/pmcab_$b/pmc$i -o pmc \
                    --output-format csv -- python3 tools/kernel_driver.py --reps 3
                i=$((i+1))
            done
            python3 tools/pmc_summary.py gpurun_out/pmcab_$b > gpurun_out/pmcab_$b.txt 2>&1
        done ;;
    pmc_era)
        # the erasure / errata kernels: the same counter groups on the driver's erasure and errata modes
        i=0
        for mode in erasure errata; do
            for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                       "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY" \
                       "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
                run pmc_${mode}_$i 300 rocprofv3 --pmc $grp -d gpurun_out/pmcera/pmc_${mode}_$i -o pmc --output-format csv -- \
                    python3 tools/kernel_driver.py --mode $mode --reps 3
                i=$((i+1))
            done
        done ;;
    pmc)
        # one rocprofv3 pass per counter group (never combined with tracing)
        i=0
        for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                   "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY" \
                   "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
                   "FETCH_SIZE" "WRITE_SIZE"; do
            run pmc$i 300 rocprofv3 --pmc $grp -d gpurun_out/pmc$i -o pmc --output-format csv -- \
                python3 tools/kernel_driver.py --reps 3
            i=$((i+1))
        done ;;
    traffic)
        # HBM bytes per codeword of each bench path: FETCH_SIZE and WRITE_SIZE
        # in separate passes per driver mode (tools/pmc_traffic.py)
        for mode in roundtrip erasure errata mixed; do
            for c in FETCH_SIZE WRITE_SIZE; do
                lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
                run traffic_${mode}_$lc 150 rocprofv3 --pmc $c -d gpurun_out/traffic/${mode}_$lc -o pmc \
                    --output-format csv -- python3 tools/kernel_driver.py --mode $mode --reps 3
            done
        done
        python3 tools/pmc_traffic.py gpurun_out/traffic --json gpurun_out/traffic_latest.json \
            > gpurun_out/traffic.txt 2>&1
        cat gpurun_out/traffic.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
