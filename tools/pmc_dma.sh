#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in build/base.so build/dma.so; do
  v=$(basename $lib .so)
  POPORON_AMD_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pd_${v} -o pmc --output-format csv -- python3 tools/exp_time.py --child > gpurun_out/pd_${v}.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for v in ("base","dma"):
    acc=defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/pd_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k=r["Kernel_Name"]
            if "lfsr" in k and ("<0" in k or "dma" in k):
                acc[k[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k,d in acc.items():
        print(v, k, {c: round(sum(x)/len(x)) for c,x in d.items()})
PY
