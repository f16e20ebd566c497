#!/usr/bin/env python3
"""Where a single general-kernel decode spends its time: per-call wall time
(ctypes) of a clean codeword (load + syndromes), of 1 error (BM over nr
iterations, one root) and of t errors, for long-root-count codes.

    python tools/gw_phases.py [--calls 200]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import libpoporon_amd as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    out = {}
    for params in ((8, 0x11D, 1, 1, 100), (8, 0x11D, 3, 1, 200), (8, 0x187, 5, 7, 48), (7, 0x89, 1, 1, 20)):
        m, poly, fcr, prim, nr = params
        nn = (1 << m) - 1
        k = nn - nr
        h = P.Poporon(*params)
        rng = np.random.default_rng(nr)
        data = rng.integers(0, nn + 1, (a.calls, k), dtype=np.uint8)
        cw = np.concatenate([data, h.encode_batch(data)], 1)
        row = {}
        for ne in (0, 1, nr // 4, nr // 2):
            bad = cw.copy()
            for c in range(a.calls):
                pos = rng.permutation(nn)[:ne]
                bad[c, pos] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
            h.decode(bad[0, :k], bad[0, k:])
            t0 = time.perf_counter()
            for c in range(a.calls):
                h.decode(bad[c, :k], bad[c, k:])
            row[f"{ne}_errors_us"] = round((time.perf_counter() - t0) / a.calls * 1e6, 1)
        out[str(params)] = row
        print(params, json.dumps(row), flush=True)
        h.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
