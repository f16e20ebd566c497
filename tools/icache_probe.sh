#!/bin/bash
# tools/icache_probe.sh LIB... -- instruction-cache counters of the kernels of
# each library build (experiments): one rocprofv3 --pmc pass per build over
# tools/exp_time.py's child workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
    v=$(basename "$lib" .so)
    POPORON_AMD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU \
        -d gpurun_out/ic_$v -o pmc --output-format csv -- python3 tools/exp_time.py --child > gpurun_out/ic_$v.log 2>&1 || exit 1
done
python3 - "$@" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
for lib in sys.argv[1:]:
    v = os.path.basename(lib)[:-3]
    acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
    for f in glob.glob(f"gpurun_out/ic_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:28]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k in acc:
        d = len(n[k]) or 1
        print(v, k, {c: round(x / d) for c, x in acc[k].items()})
PY
