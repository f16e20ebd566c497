#!/usr/bin/env python3
"""Per-call latency of the single-codeword API (poporon_encode / poporon_decode
through ctypes) for a code with fewer than 32 roots against RS(255,223).

    python tools/nr_single.py [--calls 300]"""
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
    ap.add_argument("--calls", type=int, default=300)
    a = ap.parse_args()
    out = {}
    for params in ((8, 0x11D, 1, 1, 32), (8, 0x11D, 1, 1, 16), (8, 0x11D, 1, 1, 8)):
        nr = params[4]
        k = 255 - nr
        h = P.Poporon(*params)
        rng = np.random.default_rng(nr)
        msgs = rng.integers(0, 256, (a.calls, k), dtype=np.uint8)
        h.encode(msgs[0])
        t0 = time.perf_counter()
        pars = [h.encode(m) for m in msgs]
        te = (time.perf_counter() - t0) / a.calls
        bad = []
        for m, p in zip(msgs, pars):
            cw = np.concatenate([m, p])
            pos = rng.permutation(255)[:nr // 2]
            cw[pos] ^= rng.integers(1, 256, len(pos), dtype=np.uint8)
            bad.append(cw)
        h.decode(bad[0][:k], bad[0][k:])
        t0 = time.perf_counter()
        res = [h.decode(cw[:k], cw[k:]) for cw in bad]
        td = (time.perf_counter() - t0) / a.calls
        assert all(r[0] for r in res)
        assert all((np.concatenate([r[2], r[3]]) == np.concatenate([m, p])).all() for r, m, p in zip(res, msgs, pars))
        out[f"RS(255,{k})"] = {"encode_us": round(te * 1e6, 1), "decode_t_errors_us": round(td * 1e6, 1)}
        print(f"RS(255,{k})", out[f"RS(255,{k})"], flush=True)
        h.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
