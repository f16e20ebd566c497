#!/usr/bin/env python3
"""Generate tests/golden/rng_golden.npz from the REAL reference's RNG
(src/rng.c, oracle/_ref/libpoporon_ref.so): for several seeds (none, 1-, 2-,
4- and 8-byte seeds) the bytes of consecutive poporon_rng_next calls of sizes
CALLS, concatenated.  Run here:  python tools/gen_golden_rng.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import REF_SO, reference_available  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "rng_golden.npz")
SEEDS = [b"", b"\x07", b"\x34\x12", b"\xef\xbe\xad\xde", (12345).to_bytes(4, "little"), b"\x01\x02\x03\x04\x05\x06\x07\x08"]
CALLS = [1, 3, 4, 7, 100, 4096, 5, 1 << 13]


def main():
    if not reference_available():
        sys.exit("oracle/_ref not built")
    L = C.CDLL(REF_SO)
    L.poporon_rng_create.restype = C.c_void_p
    L.poporon_rng_create.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
    L.poporon_rng_next.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.poporon_rng_next.restype = C.c_bool
    L.poporon_rng_destroy.argtypes = [C.c_void_p]
    out = {"calls": np.array(CALLS, np.uint32)}
    for i, sd in enumerate(SEEDS):
        sb = np.frombuffer(sd, np.uint8).copy() if sd else None
        h = L.poporon_rng_create(0, sb.ctypes.data_as(C.c_void_p) if sb is not None else None, len(sd))
        chunks = []
        for n in CALLS:
            b = np.zeros(n, np.uint8)
            assert L.poporon_rng_next(h, b.ctypes.data_as(C.c_void_p), n)
            chunks.append(b)
        L.poporon_rng_destroy(h)
        out[f"seed{i}"] = np.frombuffer(sd, np.uint8).copy()
        out[f"stream{i}"] = np.concatenate(chunks)
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
