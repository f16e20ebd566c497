#!/usr/bin/env python3
"""Per-stage counter deltas of the correction kernel from rocprofv3 --pmc
counter_collection CSVs written while tools/ablate_pmc.py ran.

    python tools/pmc_stages.py gpurun_out/pmcA gpurun_out/pmcB ...

Dispatches of rs_correct_k come in pairs (warm-up, measured) per stop_at in
ablate_pmc.STOPS order; the measured one of each pair is used."""
import csv
import glob
import os
import sys
from collections import defaultdict

STOPS = (1, 2, 3, 4, 0)
NAMES = {1: "syndrome load", 2: "+erasure/BM", 3: "+Omega", 4: "+Chien", 0: "+Forney/apply"}


def load(d):
    per = defaultdict(dict)  # dispatch id -> counter -> value
    kname = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "rs_correct_k" not in row.get("Kernel_Name", ""):
                continue
            did = int(row["Dispatch_Id"])
            per[did][row["Counter_Name"]] = per[did].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            kname[did] = row["Kernel_Name"]
    return [per[k] for k in sorted(per)]


def main():
    rows = defaultdict(dict)
    for d in sys.argv[1:]:
        disp = load(d)
        meas = disp[1::2]
        for stop, c in zip(STOPS, meas):
            rows[stop].update(c)
    names = sorted({k for r in rows.values() for k in r})
    print("stage".ljust(18) + "".join(n[:22].rjust(24) for n in names))
    prev = None
    for stop in STOPS:
        r = rows[stop]
        print(NAMES[stop].ljust(18) + "".join(f"{r.get(n, 0):24.0f}" for n in names))
    print("-- deltas per stage")
    prev = {}
    for stop in STOPS:
        r = rows[stop]
        print(NAMES[stop].ljust(18) + "".join(f"{r.get(n, 0) - prev.get(n, 0):24.0f}" for n in names))
        prev = r


if __name__ == "__main__":
    main()
