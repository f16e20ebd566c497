#!/usr/bin/env python3
"""Path-level roofline fractions recomputed from a rocprofv3 --kernel-trace
run of bench.py (the check on bench.py's HIP-event `roofline_modes`).

    python tools/path_roofline.py profiles/r03_kernel_trace_vN.csv [--n 1048576]

Reads the per-dispatch trace (`*_kernel_trace.csv`), orders the codec's
dispatches by start time and cuts them into path instances: an encode is one
rs_lfsr_k<0,..> dispatch; a decode starts at a remainder dispatch
(rs_lfsr_k<1,..>) and runs up to the next LFSR dispatch or non-codec kernel
(the test channel, torch).  A decode instance is decode16 when it holds
rs_bm_k, errata16e8 when its rs_ebm_k did work (> 20 us: in the erasure32
mode the errata kernels only take their early exit) and erasure32 otherwise
-- the same kernel sets bench.py sums per mode (bench.PATHS).  A path's time
is the mean over its instances of the sum of their dispatch durations;
achieved = 255 B x n / that time, frac = achieved / 8 TB/s.
(A `*_kernel_stats.csv` cannot separate rs_era_bp_k's two roles: 32 sorted
erasures in erasure32, the 16-us hand-off in errata16e8.)
"""
import argparse
import csv
import re
from collections import defaultdict

CODEC = re.compile(r"^(rs_\w+|bch\w*)")


def short(name):
    return re.sub(r"\(.*", "", re.sub(r"^void ", "", name))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--n", type=int, default=1 << 20, help="codewords per launch")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    inst = {"encode": [], "decode16": [], "erasure32": [], "errata16e8": []}
    cur = None

    def close():
        nonlocal cur
        if cur:
            names = [k for k, _ in cur]
            if any(re.match(r"rs_bm_k\b", k) for k in names):  # rs_bm_k<false> (32 roots) / <true> (fewer)
                mode = "decode16"
            elif any(k == "rs_ebm_k" and d > 20e3 for k, d in cur):
                mode = "errata16e8"
            else:
                mode = "erasure32"
            inst[mode].append(cur)
        cur = None

    for r in rows:
        k = short(r["Kernel_Name"])
        d = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        if not CODEC.match(k):
            close()
            continue
        if k.startswith("rs_lfsr_k<0"):
            close()
            inst["encode"].append([(k, d)])
        elif k.startswith("rs_lfsr_k<1"):
            close()
            cur = [(k, d)]
        elif cur is not None:
            cur.append((k, d))
    close()
    res = {}
    for mode, lst in inst.items():
        if not lst:
            continue
        per = defaultdict(float)
        for one in lst:
            for k, d in one:
                per[k] += d / len(lst)
        tot = sum(per.values())
        gbs = 255 * a.n / (tot * 1e-9) / 1e9
        res[mode] = tot
        print(f"{mode:10s} path {tot / 1e3:8.1f} us  {gbs:8.1f} GB/s  frac {gbs / 8000:.4f}  ({len(lst)} launch sets) [" +
              ", ".join(f"{k} {v / 1e3:.1f}us" for k, v in per.items()) + "]")
    if "encode" in res and "decode16" in res:
        t = res["encode"] + res["decode16"]
        gbs = 2 * 255 * a.n / (t * 1e-9) / 1e9
        print(f"{'roundtrip':10s} path {t / 1e3:8.1f} us  {gbs:8.1f} GB/s  frac {gbs / 8000:.4f}")


if __name__ == "__main__":
    main()
