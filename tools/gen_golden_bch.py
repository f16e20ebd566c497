#!/usr/bin/env python3
"""Generate tests/golden/bch_golden.npz by running the REAL reference's BCH codec.

SURVEY.md 8(f) rank 4 (BCH reuses the GF tables).  For each parameter set
(symbol_size 3..5: codewords of up to 31 bits, where the reference's uint32
arithmetic is defined) it records, from ``oracle/_ref/libpoporon_ref.so``
(compiled from /root/reference/src by oracle/Makefile) driven through
poporon_bch_config_create / poporon_create / poporon_encode / poporon_decode:

  enc_*  every message value (or 512 random ones) -> parity bytes
  dec_*  received words with 0 .. t+3 flipped bits over data and parity,
         data bits above the message length set in some inputs; the result
         bool, corrected_num (a sentinel 777 is passed in: the reference leaves
         it untouched on failure) and the data bytes out
Also the getters (parity / info sizes).

Run here (not on the GPU box):  python tools/gen_golden_bch.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ReferenceBch, reference_available  # noqa: E402

SEED = 0x5EED0003
OUT = os.path.join(ROOT, "tests", "golden", "bch_golden.npz")
PARAMS = [(4, 0x13, 3), (4, 0x13, 1), (4, 0x13, 2), (3, 0x0B, 1), (3, 0x0B, 2), (5, 0x25, 1), (5, 0x25, 2),
          (5, 0x25, 3), (5, 0x25, 5), (5, 0x25, 7), (4, 0x19, 2), (5, 0x3D, 4)]
SENT = 777


def main():
    if not reference_available():
        sys.exit("oracle/_ref/libpoporon_ref.so missing: run `make -C oracle` with /root/reference present")
    rng = np.random.default_rng(SEED)
    out = {"params": np.array(PARAMS, np.uint16)}
    for gi, (m, poly, t) in enumerate(PARAMS):
        ref = ReferenceBch(m, poly, t)
        pb, ib = ref.parity_bytes, ref.info_bytes
        pre = f"b{gi}_"
        out[pre + "sizes"] = np.array([pb, ib], np.uint32)
        # messages: ib bytes (random bytes, including bits above k)
        nmsg = 512
        msgs = rng.integers(0, 256, (nmsg, max(ib, 1)), dtype=np.uint8)[:, :ib]
        par = np.zeros((nmsg, max(pb, 1)), np.uint8)
        for i in range(nmsg):
            ok, p = ref.encode(msgs[i])
            assert ok
            par[i, :pb] = p
        out[pre + "enc_data"], out[pre + "enc_parity"] = msgs, par
        # decodes: flip bits of the (data, parity) byte images
        ndec = 600
        din = np.zeros((ndec, max(ib, 1)), np.uint8)
        pin = np.zeros((ndec, max(pb, 1)), np.uint8)
        dout = np.zeros((ndec, max(ib, 1)), np.uint8)
        dok = np.zeros(ndec, np.uint8)
        dcor = np.zeros(ndec, np.uint32)
        nerr = np.zeros(ndec, np.uint8)
        for i in range(ndec):
            j = int(rng.integers(0, nmsg))
            d, p = msgs[j].copy(), par[j, :pb].copy()
            e = int(rng.integers(0, t + 4))
            nerr[i] = e
            din[i, :ib], pin[i, :pb] = d, p
            # flip bits in the byte images directly: bit positions over all data and parity bytes
            allbits = rng.permutation(8 * (ib + pb))[:e]
            for b in allbits:
                if b < 8 * ib:
                    din[i, b // 8] ^= np.uint8(1 << (b % 8))
                else:
                    c = b - 8 * ib
                    pin[i, c // 8] ^= np.uint8(1 << (c % 8))
            ok, cor, dd = ref.decode(din[i, :ib], pin[i, :pb], SENT)
            dout[i, :ib] = dd
            dok[i], dcor[i] = ok, cor
        out[pre + "dec_data"], out[pre + "dec_parity"] = din, pin
        out[pre + "dec_out"], out[pre + "dec_ok"], out[pre + "dec_cor"] = dout, dok, dcor
        out[pre + "dec_nerr"] = nerr
        print(f"set {gi} {PARAMS[gi]}: parity {pb} B, info {ib} B, {int(dok.sum())}/{ndec} decodes ok")
        ref.close()
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
