#!/usr/bin/env python3
"""Path-level roofline fractions recomputed from a rocprofv3 --kernel-trace
--stats CSV (the check on bench.py's HIP-event `roofline_modes`).

    python tools/path_roofline.py profiles/r03_kernel_stats_vN.csv [--n 1048576]

A path's time per launch-set is the sum of its kernels' average dispatch
durations; achieved = 255 B x n / that time; frac = achieved / 8 TB/s.
"""
import argparse
import csv
import re

MODES = {
    "encode": [r"rs_lfsr_k<0,"],
    "decode16": [r"rs_lfsr_k<1,", r"^rs_bm_k\(", r"^rs_chien_k\(", r"rs_forney_k", r"rs_apply_k<16>",
                 r"rs_correct_k<unsigned char, false, false>"],
    "erasure32": [r"rs_lfsr_k<1,", r"^rs_era_k\(", r"rs_correct_k<unsigned char, true, true>", r"rs_apply_k<32>"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--n", type=int, default=1 << 20, help="codewords per launch")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    for name in rows:
        name["Name"] = re.sub(r"^void ", "", name["Name"])
    res = {}
    for mode, pats in MODES.items():
        tot, parts = 0.0, []
        for p in pats:
            hit = [r for r in rows if re.search(p, r["Name"])]
            if not hit:
                continue
            ns = sum(float(r["TotalDurationNs"]) for r in hit) / sum(int(r["Calls"]) for r in hit)
            tot += ns
            parts.append(f"{hit[0]['Name'].split('(')[0]} {ns / 1e3:.1f}us")
        if tot:
            gbs = 255 * a.n / (tot * 1e-9) / 1e9
            res[mode] = tot
            print(f"{mode:10s} path {tot / 1e3:8.1f} us  {gbs:8.1f} GB/s  frac {gbs / 8000:.4f}   [" +
                  ", ".join(parts) + "]")
    if "encode" in res and "decode16" in res:
        t = res["encode"] + res["decode16"]
        gbs = 2 * 255 * a.n / (t * 1e-9) / 1e9
        print(f"{'roundtrip':10s} path {t / 1e3:8.1f} us  {gbs:8.1f} GB/s  frac {gbs / 8000:.4f}")


if __name__ == "__main__":
    main()
