#!/usr/bin/env python3
"""HBM traffic per codeword of each bench path, from rocprofv3 --pmc passes.

    python tools/pmc_traffic.py gpurun_out/traffic --json profiles/traffic_latest.json

Expects <dir>/<mode>_fetch/*counter_collection.csv and <dir>/<mode>_write/...
for mode in {roundtrip, erasure, errata, mixed}: one `rocprofv3 --pmc FETCH_SIZE` and one
`--pmc WRITE_SIZE` pass (never together with tracing; tools/gpu_session.sh
step `traffic`) over `tools/kernel_driver.py --mode <mode> --n N`.

Per kernel dispatch (MI355X_MICROARCH.md "HBM"):
    read bytes  = FETCH_SIZE (KB) x 1024 x 2   (gfx950 counts 1/2 of wide reads)
    write bytes = WRITE_SIZE (KB) x 1024
averaged over the dispatches of each kernel, divided by the codewords of a
dispatch, and summed over the kernels of each bench path (bench.PATHS):
encode (roundtrip run), decode16 (roundtrip run), erasure32 (erasure run),
errata16e8 (errata run).
The output is stamped with bench.source_stamp(): bench.py ignores a file
whose stamp does not match the kernel sources it runs.
"""
import argparse
import csv
import datetime
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

# rocprof kernel name -> bench kernel id (include/poporon_amd.h)
PATTERNS = [
    (r"rs_lfsr_k<0,", bench.K_ENCODE), (r"rs_lfsr_k<1,", bench.K_REMAINDER),
    (r"\brs_bm_k\b|\brs_ebm_k\b", bench.K_BM), (r"\brs_chien_k\b|\brs_chien32_k\b", bench.K_CHIEN),
    (r"rs_forney_k|rs_forney32_k", bench.K_FORNEY),
    (r"rs_apply_k", bench.K_APPLY), (r"\brs_era_bp_k\b|\brs_era_k\b", bench.K_ERASURE),
    (r"\brs_wave_k\b|\brs_list1_k\b|rs_correct_k<[^>]*true>|rs_correct_list|rs_correct_k", bench.K_LIST),
]


def kernel_id(name):
    for pat, k in PATTERNS:
        if re.search(pat, name):
            return k
    return None


def read_pass(d, counter):
    """{kernel id: average counter value per dispatch}"""
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = kernel_id(row["Kernel_Name"])
            if k is not None:
                acc[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--n", type=int, default=1 << 20, help="codewords per dispatch (kernel_driver --n)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    runs = {"encode": "roundtrip", "decode16": "roundtrip", "erasure32": "erasure", "errata16e8": "errata",
            "decode_mixed": "mixed"}
    out = {"source_stamp": bench.source_stamp(), "date": datetime.datetime.utcnow().strftime("%Y-%m-%d %H:%M UTC"),
           "codewords_per_dispatch": a.n,
           "note": "hbm bytes = FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 per dispatch (MI355X_MICROARCH.md HBM; the "
                   "x2 read correction is calibrated for 16-B coalesced loads), averaged over dispatches, per codeword, "
                   "summed over the path's kernels", "modes": {}}
    for mode, run in runs.items():
        fetch, nf = read_pass(os.path.join(a.dir, f"{run}_fetch"), "FETCH_SIZE")
        write, nw = read_pass(os.path.join(a.dir, f"{run}_write"), "WRITE_SIZE")
        ks = [k for k in bench.PATHS[mode] if k in fetch and k in write]
        if not ks:
            continue
        per = {}
        for k in ks:
            rd, wr = fetch[k] * 1024 * 2, write[k] * 1024
            per[str(k)] = {"read_bytes_per_cw": round(rd / a.n, 2), "write_bytes_per_cw": round(wr / a.n, 2),
                           "dispatches": nf[k]}
        tot = sum(v["read_bytes_per_cw"] + v["write_bytes_per_cw"] for v in per.values())
        out["modes"][mode] = {"hbm_bytes_per_cw": round(tot, 2), "ratio_to_255": round(tot / bench.CW_BYTES, 3),
                              "kernels": per}
        print(f"{mode:10s} {tot:8.1f} B/cw  ({tot / bench.CW_BYTES:.2f} x 255)  " +
              "  ".join(f"{k}:{v['read_bytes_per_cw']:.0f}r+{v['write_bytes_per_cw']:.0f}w" for k, v in per.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
