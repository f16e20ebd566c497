#!/bin/bash
# tools/pmc_variants.sh LIB... -- one rocprofv3 --pmc pass per counter group over
# tools/exp_time.py's child workload for each library build (experiments);
# prints per-kernel averages.  Never combined with tracing (gpurun rule).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
    v=$(basename "$lib" .so)
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
               "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"; do
        POPORON_AMD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pv_${v}_$i -o pmc \
            --output-format csv -- python3 tools/exp_time.py --child > gpurun_out/pv_${v}_$i.log 2>&1 || exit 1
        i=$((i+1))
    done
done
python3 - "$@" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
for lib in sys.argv[1:]:
    v = os.path.basename(lib)[:-3]
    acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(f"gpurun_out/pv_{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:24]
            if not k.startswith("rs_"):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    for k in sorted(acc):
        print(v, k, {c: round(x / max(1, len(n[k][c]))) for c, x in sorted(acc[k].items())})
PY
