#!/usr/bin/env python3
"""Generate tests/golden/rs_params_golden.npz by running the REAL reference.

Companion of tools/gen_golden.py (RS(255,223) fixtures) for the general RS
parameters that SURVEY.md 8(f) ranks first: symbol sizes 2..8, num_roots
from 2 to 200, other field polynomials, fcr and prim (including an fcr*prim
large enough to wrap the reference's uint16 exponent arithmetic).  For each
parameter set it records, from ``oracle/_ref/libpoporon_ref.so`` (compiled
from /root/reference/src by oracle/Makefile) driven through its public API:

  enc_*  encodes at full and shortened sizes (data bytes are NOT masked to
         the symbol size: the reference masks them itself, src/encode.c:126)
  dec_*  decodes with 0 .. t+3 random errors of random magnitude over data
         and parity (failures and miscorrections included), with some data
         bits above the symbol size set (ignored by the syndromes, kept)
  era_*  erasure decodes: e <= num_roots sorted positions (+ a few errors)
  xs_*   external-syndrome decodes (config "syndrome" pointer)

Run here (not on the GPU box):  python tools/gen_golden_params.py
Deterministic: every case derives from SEED.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import Reference, reference_available  # noqa: E402

SEED = 0x5EED0002
OUT = os.path.join(ROOT, "tests", "golden", "rs_params_golden.npz")
W = 255  # row width of the stored codewords

# (symbol_size, field polynomial, fcr, prim, num_roots)
PARAMS = [
    (8, 0x11D, 1, 1, 16),      # RS(255,239)
    (8, 0x11D, 0, 1, 2),       # 2 roots
    (8, 0x187, 5, 7, 48),      # other polynomial, prim 7
    (8, 0x11D, 1, 1, 100),
    (8, 0x11D, 3, 1, 200),
    (8, 0x11D, 2000, 37, 32),  # 32 roots but (fcr+31)*prim overflows uint16: general kernels
    (7, 0x89, 1, 1, 20),       # GF(128)
    (6, 0x43, 1, 1, 10),       # GF(64)
    (5, 0x25, 3, 1, 6),        # GF(32)
    (4, 0x13, 1, 2, 8),        # GF(16), prim 2
    (4, 0x13, 0, 1, 4),        # RS(15,11)
    (3, 0x0B, 1, 1, 4),        # GF(8)
    (2, 0x07, 1, 1, 2),        # GF(4)
]


def corrupt(rng, cw, L, nerr, nn):
    pos = rng.permutation(L)[:nerr]
    cw[pos] ^= rng.integers(1, nn + 1, nerr).astype(np.uint8)
    return pos


def main():
    if not reference_available():
        sys.exit("oracle/_ref/libpoporon_ref.so missing: run `make -C oracle` in the container with /root/reference")
    rng = np.random.default_rng(SEED)
    out = {"params": np.array(PARAMS, np.uint16)}
    for gi, (m, poly, fcr, prim, nr) in enumerate(PARAMS):
        nn = (1 << m) - 1
        k = nn - nr
        t = nr // 2
        ref = Reference(m, poly, fcr, prim, nr)
        pre = f"g{gi}_"

        # ---- encodes
        sizes = [k] * 24 + [int(x) for x in rng.integers(1, k + 1, 16)]
        ed = np.zeros((len(sizes), W), np.uint8)
        ep = np.zeros((len(sizes), nr), np.uint8)
        for i, s in enumerate(sizes):
            d = rng.integers(0, 256, s, dtype=np.uint8)
            ok, par = ref.encode(d)
            assert ok
            ed[i, :s], ep[i] = d, par
        out[pre + "enc_size"] = np.array(sizes, np.uint16)
        out[pre + "enc_data"], out[pre + "enc_parity"] = ed, ep

        # ---- decodes: 0 .. t+3 errors, full and shortened sizes
        cases = []
        for ne in range(0, t + 4):
            reps = 6 if ne <= t else 4
            for _ in range(reps):
                cases.append((k if rng.random() < 0.7 else int(rng.integers(1, k + 1)), ne))
        di = np.zeros((len(cases), W), np.uint8)
        do = np.zeros((len(cases), W), np.uint8)
        dok = np.zeros(len(cases), np.uint8)
        dcor = np.zeros(len(cases), np.uint32)
        for i, (s, ne) in enumerate(cases):
            d = rng.integers(0, nn + 1, s, dtype=np.uint8)
            _, par = ref.encode(d)
            cw = np.concatenate([d, par])
            corrupt(rng, cw, s + nr, min(ne, s + nr), nn)
            if m < 8 and i % 5 == 0:  # bits above the symbol size: masked by the syndromes, kept in the output
                cw[: s] |= np.uint8(0x80)
            ok, n, dd, pp = ref.decode(cw[:s], cw[s:])
            di[i, : s + nr] = cw
            do[i, : s + nr] = np.concatenate([dd, pp])
            dok[i], dcor[i] = ok, n
        out[pre + "dec_size"] = np.array([c[0] for c in cases], np.uint16)
        out[pre + "dec_nerr"] = np.array([c[1] for c in cases], np.uint16)
        out[pre + "dec_in"], out[pre + "dec_out"] = di, do
        out[pre + "dec_ok"], out[pre + "dec_cor"] = dok, dcor
        ref.close()

        # ---- erasures (sorted positions in data) + a few errors
        refe = Reference(m, poly, fcr, prim, nr, erasure=True)
        n_era = 24
        es = np.zeros(n_era, np.uint16)
        ec = np.zeros(n_era, np.uint32)
        eslots = np.zeros((n_era, nr), np.uint32)
        ei = np.zeros((n_era, W), np.uint8)
        eo = np.zeros((n_era, W), np.uint8)
        eok = np.zeros(n_era, np.uint8)
        ecor = np.zeros(n_era, np.uint32)
        for i in range(n_era):
            s = k
            e = int(rng.integers(1, min(nr, s) + 1))
            d = rng.integers(0, nn + 1, s, dtype=np.uint8)
            _, par = refe.encode(d)
            cw = np.concatenate([d, par])
            pos = np.sort(rng.permutation(s)[:e])
            cw[pos] ^= rng.integers(1, nn + 1, e).astype(np.uint8)
            x = int(rng.integers(0, max(1, (nr - e) // 2 + 2)))
            if x:
                corrupt(rng, cw, s + nr, x, nn)
            slots = np.zeros(nr, np.uint32)
            slots[:e] = pos
            refe.set_erasures(slots)  # capacity >= nr: stale slots past e are these values (quirk Q2)
            refe.set_erasures(pos)
            ok, n, dd, pp = refe.decode(cw[:s], cw[s:])
            es[i], ec[i], eslots[i] = s, e, slots
            ei[i, : s + nr] = cw
            eo[i, : s + nr] = np.concatenate([dd, pp])
            eok[i], ecor[i] = ok, n
        refe.close()
        out[pre + "era_size"], out[pre + "era_count"], out[pre + "era_slots"] = es, ec, eslots
        out[pre + "era_in"], out[pre + "era_out"], out[pre + "era_ok"], out[pre + "era_cor"] = ei, eo, eok, ecor

        # ---- external syndromes: the syndromes of a corrupted word (log form),
        # all-zero ones, and one with a single changed value
        n_xs = 6
        xs = np.zeros((n_xs, nr), np.uint16)
        xi = np.zeros((n_xs, W), np.uint8)
        xo = np.zeros((n_xs, W), np.uint8)
        xok = np.zeros(n_xs, np.uint8)
        xcor = np.zeros(n_xs, np.uint32)
        probe = Reference(m, poly, fcr, prim, nr)
        for i in range(n_xs):
            d = rng.integers(0, nn + 1, k, dtype=np.uint8)
            _, par = probe.encode(d)
            cw = np.concatenate([d, par])
            corrupt(rng, cw, k + nr, int(rng.integers(1, t + 1)), nn)
            probe.decode(cw[:k], cw[k:])  # fills the handle's syndrome scratch
            syn = probe.last_syndrome()
            if i == 0:
                syn[:] = nn
            elif i == 1:
                syn[0] = (int(syn[0]) + 1) % nn
            rx = Reference(m, poly, fcr, prim, nr, ext_syn=syn)
            ok, n, dd, pp = rx.decode(cw[:k], cw[k:])
            rx.close()
            xs[i] = syn
            xi[i, : k + nr] = cw
            xo[i, : k + nr] = np.concatenate([dd, pp])
            xok[i], xcor[i] = ok, n
        probe.close()
        out[pre + "xs_syn"], out[pre + "xs_in"], out[pre + "xs_out"] = xs, xi, xo
        out[pre + "xs_ok"], out[pre + "xs_cor"] = xok, xcor
        print(f"set {gi} {PARAMS[gi]}: {len(sizes)} enc, {len(cases)} dec ({int(dok.sum())} ok), "
              f"{n_era} era ({int(eok.sum())} ok), {n_xs} ext-syn")
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
