#!/usr/bin/env python3
"""Summarise rocprofv3 output for the rs_* kernels.

    python tools/pmc_summary.py gpurun_out [--json profiles/traffic_latest.json]

Reads <dir>/prof/*kernel_stats.csv (kernel trace --stats) and every
<dir>/pmc*/pmc_counter_collection.csv (one --pmc pass each), averages each
counter per dispatch of every rs_* kernel, and derives HBM traffic per launch:
  read bytes  = FETCH_SIZE (KB) * 1024 * 2   (gfx950 reports 1/2 of the bytes
                of wide streaming reads, MI355X_MICROARCH.md "HBM")
  write bytes = WRITE_SIZE (KB) * 1024
The x2 read correction is calibrated for 16-B/lane coalesced loads only;
the LFSR kernels load 4 B/lane at a 255-B lane stride, so the read figure is
an estimate (noted in the JSON).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

NAMES = {"rs_lfsr_k<0>": "rs_lfsr_k<false> (encode)", "rs_lfsr_k<1>": "rs_lfsr_k<true> (remainder)",
         "rs_lfsr_k<2>": "rs_lfsr_k (check)", "rs_correct_k<unsigned char>": "rs_correct_k (BM/Chien/Forney)",
         "rs_correct_k<unsigned int>": "rs_correct_k (BM/Chien/Forney, u32 slots)",
         # template <MODE, PATH> / <PosT, ERA> names of the current kernels (bench.py's keys)
         "rs_lfsr_k<0, 0>": "rs_lfsr_k<false> (encode)", "rs_lfsr_k<0, 1>": "rs_lfsr_k<false> (encode)",
         "rs_lfsr_k<1, 2>": "rs_lfsr_k<true> (remainder)", "rs_lfsr_k<1, 1>": "rs_lfsr_k<true> (remainder)",
         "rs_correct_k<unsigned char, false>": "rs_correct_k (BM/Chien/Forney)",
         "rs_correct_k<unsigned char, true>": "rs_correct_k (erasure, u8 slots)",
         "rs_correct_k<unsigned int, true>": "rs_correct_k (erasure, u32 slots)",
         "rs_bm_k": "rs_bm_k (BM/Omega)", "rs_chien_k": "rs_chien_k (Chien)",
         "rs_forney_k": "rs_forney_k (Forney)", "rs_apply_k": "rs_apply_k (apply)"}


def short(name):
    m = re.search(r"(rs_[a-z_]+<[^>]*>)", name)
    if m:
        return m.group(1)
    m = re.search(r"\b(rs_(?:bm|bmp|chien|forney|apply|era_bp|ebm|chien32|forney32)_k)\b", name)
    return m.group(1) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = {}
    for f in glob.glob(os.path.join(a.dir, "prof", "*kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            k = short(row["Name"])
            if k:
                out.setdefault(k, {})["avg_ns"] = float(row["AverageNs"])
                out[k]["calls"] = int(row["Calls"])
                print(f"{k:32s} calls {row['Calls']:>4s}  avg {float(row['AverageNs'])/1e3:9.1f} us")
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(a.dir, "pmc*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            if not k:
                continue
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            meta[k] = (row["VGPR_Count"], row["SGPR_Count"], row["LDS_Block_Size"], row["Scratch_Size"])
    for k, cs in acc.items():
        print(f"\n{k}  vgpr/sgpr/lds/scratch = {meta[k]}")
        for c in sorted(cs):
            v = cs[c]
            print(f"   {c:24s} {sum(v)/len(v):16.1f}   (n={len(v)})")
        d = out.setdefault(k, {})
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d["counters"] = avg
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            d["hbm_bytes_per_launch"] = avg["FETCH_SIZE"] * 1024 * 2 + avg["WRITE_SIZE"] * 1024
            d["fetch_kb_raw"] = avg["FETCH_SIZE"]
            d["write_kb"] = avg["WRITE_SIZE"]
        if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
            d["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
    if a.json:
        kernels = {NAMES.get(k, k): v for k, v in out.items()}
        with open(a.json, "w") as f:
            json.dump({"source": a.dir, "note": "hbm_bytes_per_launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 "
                       "(read doubling calibrated for 16-B coalesced loads only)", "kernels": kernels}, f, indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
