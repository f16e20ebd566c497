#!/usr/bin/env python3
"""Single-codeword poporon_decode calls (16 errors) in a loop, for a
rocprofv3 kernel trace of the drop-in calling pattern."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import libpoporon_amd as P  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rs = P.Poporon.default()
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 223, dtype=np.uint8)
    par = rs.encode(data)
    cw = np.concatenate([data, par])
    bad = cw.copy()
    pos = rng.permutation(255)[:16]
    bad[pos] ^= rng.integers(1, 256, 16, dtype=np.uint8)
    for _ in range(20):
        rs.decode(bad[:223].copy(), bad[223:].copy())
    t0 = time.perf_counter()
    for _ in range(n):
        r = rs.decode(bad[:223].copy(), bad[223:].copy())
    dt = (time.perf_counter() - t0) / n
    assert r[0] and r[1] == 16 and (np.concatenate([r[2], r[3]]) == cw).all()
    print(f"decode16 {dt * 1e6:.1f} us per call ({os.environ.get('POPORON_AMD_DECODE_PATH', 'default')})")


if __name__ == "__main__":
    main()
