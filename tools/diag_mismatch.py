#!/usr/bin/env python3
"""Diagnose GPU-vs-oracle decode mismatches on random batches (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import libpoporon_amd as P  # noqa: E402
from oracle import Oracle  # noqa: E402


def run(label, nerr_fn, n=4096, seed=1):
    o = Oracle()
    h = P.Poporon.default()
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (n, 223), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    ne = np.array([nerr_fn(c, rng) for c in range(n)])
    for c in range(n):
        pos = rng.permutation(255)[: ne[c]]
        cw[c, pos] ^= rng.integers(1, 256, ne[c], dtype=np.uint8)
    ok, cor, d, p = h.decode_batch(cw[:, :223], cw[:, 223:])
    ook, ocor, od, op = o.decode_batch(cw[:, :223], cw[:, 223:])
    bad = np.nonzero((ok != ook) | (cor != ocor) | (d != od).any(1) | (p != op).any(1))[0]
    print(f"{label}: {len(bad)} / {n} mismatches")
    for c in bad[:12]:
        w = c // 64
        wave_ne = ne[w * 64:(w + 1) * 64]
        print(f"  cw {c} ne={ne[c]} gpu ok={ok[c]} cor={cor[c]} | ora ok={ook[c]} cor={ocor[c]} "
              f"bytes_diff={(d[c] != od[c]).sum() + (p[c] != op[c]).sum()} wave max ne={wave_ne.max()} "
              f"min ne={wave_ne.min()}")


if __name__ == "__main__":
    run("all 16", lambda c, r: 16)
    run("0..16", lambda c, r: int(r.integers(0, 17)))
    run("1..16", lambda c, r: int(r.integers(1, 17)))
    run("16 + one 20 per wave", lambda c, r: 20 if c % 64 == 5 else 16)
    run("8 + zeros", lambda c, r: 8 if c % 2 else 0)
    run("0..20", lambda c, r: int(r.integers(0, 21)))
