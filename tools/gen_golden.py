#!/usr/bin/env python3
"""Generate tests/golden/rs255_golden.npz by running the REAL reference.

The reference (libpoporon, /root/reference) ships no golden vectors for RS
(its tests are time-seeded and use 0xFF magnitudes, tests/util.h:20-94), so
this script makes them: it loads ``oracle/_ref/libpoporon_ref.so`` (compiled
from /root/reference/src by ``oracle/Makefile``) and records inputs and the
reference's outputs for every behaviour class of SURVEY.md section 8(c).
Only the reference's public API is driven, except for reading the GF tables,
the generator and the handle's syndrome scratch through a struct mirror
(oracle.Reference.rs_tables / last_syndrome).

Run here (not on the GPU box):  python tools/gen_golden.py
Deterministic: every case derives from SEED.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import Reference, reference_available  # noqa: E402

SEED = 0x5EED0001
OUT = os.path.join(ROOT, "tests", "golden", "rs255_golden.npz")
NR = 32


def main():
    if not reference_available():
        sys.exit("oracle/_ref/libpoporon_ref.so missing: run `make -C oracle` in the container with /root/reference")
    rng = np.random.default_rng(SEED)
    out = {}

    # ---- GF tables / generator / primitive inverse for several parameter sets
    params = [(8, 0x11D, 1, 1, 32), (8, 0x11D, 0, 1, 32), (8, 0x11D, 2, 1, 32), (8, 0x11D, 1, 2, 32),
              (8, 0x11D, 1, 1, 16), (8, 0x187, 1, 1, 32), (8, 0x11D, 112, 11, 32), (4, 0x13, 1, 2, 8)]
    out["param_sets"] = np.array(params, np.uint16)
    for i, p in enumerate(params):
        r = Reference(*p)
        alog, log, gen, iprim = r.rs_tables()
        out[f"p{i}_alog"], out[f"p{i}_log"], out[f"p{i}_gen"] = alog, log, gen
        out[f"p{i}_iprim"] = np.array([iprim], np.uint16)
        r.close()
    ref = Reference()
    out["gf_mod_in"] = np.array([0, 1, 254, 255, 256, 257, 510, 511, 4096, 8128, 65535], np.uint16)
    gfh = ref.lib.poporon_gf_create(8, 0x11D)
    out["gf_mod_out"] = np.array([ref.lib.poporon_gf_mod(gfh, int(v)) for v in out["gf_mod_in"]], np.uint8)
    ref.lib.poporon_gf_destroy(gfh)
    out["version_id"] = np.array([ref.lib.poporon_version_id()], np.uint32)

    # ---- encode: full-size and shortened messages
    sizes = [223] * 768 + [1] * 16 + [64] * 64 + [100] * 32 + [222] * 32 + [2] * 16
    enc_data = np.zeros((len(sizes), 223), np.uint8)
    enc_par = np.zeros((len(sizes), NR), np.uint8)
    for i, s in enumerate(sizes):
        d = rng.integers(0, 256, s, dtype=np.uint8)
        if i == 0:
            d = np.arange(223, dtype=np.uint8)
        elif i == 1:
            d = np.zeros(223, np.uint8)
        elif i == 2:
            d = np.full(223, 0xFF, np.uint8)
        enc_data[i, :s] = d
        ok, enc_par[i] = ref.encode(d)
        assert ok
    out["enc_size"], out["enc_data"], out["enc_parity"] = np.array(sizes, np.uint16), enc_data, enc_par

    # ---- decode without erasures: 0..25 random-magnitude errors over data AND parity
    cases = []

    def dec_case(size, ne, kind, mags=None):
        d = rng.integers(0, 256, size, dtype=np.uint8)
        _, p = ref.encode(d)
        cw = np.concatenate([d, p])
        pos = rng.permutation(size + NR)[:ne]
        if mags is None:
            mags = rng.integers(1, 256, ne, dtype=np.uint8)
        cw[pos] ^= mags
        ok, n, od, op = ref.decode(cw[:size], cw[size:])
        syn = ref.last_syndrome()
        return dict(size=size, ne=ne, kind=kind, inp=cw, ok=ok, cor=n, out=np.concatenate([od, op]), syn=syn,
                    clean=np.concatenate([d, p]))

    for ne in list(range(0, 17)):
        for _ in range(48 if ne in (0, 1, 8, 15, 16) else 24):
            cases.append(dec_case(223, ne, 0))
    for ne in (1, 4, 16):  # reference's own magnitude: 0xFF (tests/util.h:51)
        for _ in range(8):
            cases.append(dec_case(223, ne, 1, mags=np.full(ne, 0xFF, np.uint8)))
    for size in (1, 2, 64, 100, 222):  # shortened codes (pad > 0)
        for ne in (0, 1, 5, 16, 17, 20):
            for _ in range(6):
                cases.append(dec_case(size, ne, 2) if ne <= size + NR else None)
    cases = [c for c in cases if c is not None]
    # beyond capacity, random patterns: the reference fails them (no random
    # miscorrection shows up in 15k trials), so record a sample of failures ...
    fails = [dec_case(223, int(rng.integers(17, 26)), 3) for _ in range(160)]
    # ... and construct miscorrections: g(x)*x^s is a weight-33 codeword, so
    # flipping ne >= 17 of its nonzero symbols leaves the word 33-ne <= 16 away
    # from the neighbouring codeword, which the decoder then "corrects" to.
    _, _, gen_log, _ = ref.rs_tables()
    alog = ref.rs_tables()[0]
    gpoly = alog[gen_log].astype(np.uint8)  # poly form, gpoly[i] = coeff of x^i
    misc = []
    for k in range(48):
        ne = 17 + k % 8
        d = rng.integers(0, 256, 223, dtype=np.uint8)
        _, p = ref.encode(d)
        clean = np.concatenate([d, p])
        s = int(rng.integers(0, 255 - 32))
        cw_g = np.zeros(255, np.uint8)  # index 0 = x^254
        for i in range(33):
            cw_g[254 - (i + s)] = gpoly[i]
        scale = int(rng.integers(1, 256))  # any nonzero multiple is a codeword too
        log_tab = ref.rs_tables()[1]
        cw_g = np.array([0 if v == 0 else alog[(int(log_tab[v]) + int(log_tab[scale])) % 255] for v in cw_g], np.uint8)
        supp = np.nonzero(cw_g)[0]
        flip = rng.permutation(supp)[:ne]
        cw = clean.copy()
        cw[flip] ^= cw_g[flip]
        ok, n, od, op = ref.decode(cw[:223], cw[223:])
        misc.append(dict(size=223, ne=ne, kind=4, inp=cw, ok=ok, cor=n, out=np.concatenate([od, op]),
                         syn=ref.last_syndrome(), clean=clean))
    assert sum(c["ok"] for c in misc) > 0
    cases += misc + fails
    n = len(cases)
    out["dec_size"] = np.array([c["size"] for c in cases], np.uint16)
    out["dec_nerr"] = np.array([c["ne"] for c in cases], np.uint16)
    out["dec_kind"] = np.array([c["kind"] for c in cases], np.uint8)
    out["dec_in"] = np.zeros((n, 255), np.uint8)
    out["dec_out"] = np.zeros((n, 255), np.uint8)
    out["dec_clean"] = np.zeros((n, 255), np.uint8)
    out["dec_syn"] = np.stack([c["syn"] for c in cases]).astype(np.uint16)
    for i, c in enumerate(cases):
        L = c["size"] + NR
        out["dec_in"][i, :L] = c["inp"]
        out["dec_out"][i, :L] = c["out"]
        out["dec_clean"][i, :L] = c["clean"]
    out["dec_ok"] = np.array([c["ok"] for c in cases], np.uint8)
    out["dec_cor"] = np.array([c["cor"] for c in cases], np.uint32)

    # ---- erasure decode: the erasure object's slots beyond the count are
    # pre-filled (add 32 stale positions, reset, add the real ones) so that the
    # reference's slot-by-root-index apply (quirks Q1/Q2/Q3) is deterministic.
    eref = Reference(erasure=True)
    ecases = []

    def eras_case(size, e, extra_err, sort, kind, mags=None, stale=None):
        d = rng.integers(0, 256, size, dtype=np.uint8)
        _, p = eref.encode(d)
        cw = np.concatenate([d, p])
        perm = rng.permutation(size)  # erasures inside data[] (parity erasures are UB, Q4)
        epos = perm[:e]
        if sort:
            epos = np.sort(epos)
        if stale is None:
            stale = rng.permutation(size)[:NR] if size >= NR else rng.integers(0, size, NR)
        slots = np.array(stale, np.uint32)
        slots[:e] = epos
        if mags is None:
            mags = rng.integers(1, 256, e, dtype=np.uint8)
        cw[epos] ^= mags
        rest = np.setdiff1d(np.arange(size + NR), epos)
        xpos = rng.permutation(rest)[:extra_err]
        cw[xpos] ^= rng.integers(1, 256, extra_err, dtype=np.uint8)
        eref.set_erasures(stale)
        eref.set_erasures(epos)
        ok, n, od, op = eref.decode(cw[:size], cw[size:])
        return dict(size=size, e=e, x=extra_err, kind=kind, slots=slots, inp=cw, ok=ok, cor=n,
                    out=np.concatenate([od, op]), clean=np.concatenate([d, p]))

    for _ in range(64):
        ecases.append(eras_case(223, 32, 0, True, 0))            # config 4
    for _ in range(32):
        ecases.append(eras_case(223, 32, 0, False, 1))           # Q1
    for e in (1, 2, 8, 16, 24, 31):
        for _ in range(8):
            ecases.append(eras_case(223, e, 0, True, 2))
            ecases.append(eras_case(223, e, 0, False, 2))
    for _ in range(16):
        ecases.append(eras_case(64, 16, 0, False, 3, mags=np.full(16, 0xFF, np.uint8)))  # tests/test_codec.c:123-168
        ecases.append(eras_case(64, 20, 0, False, 3, mags=np.full(20, 0xFF, np.uint8)))  # tests/test_unified.c:82-112
    for e, x in ((8, 4), (16, 8), (2, 15), (20, 6), (10, 12)):
        for _ in range(8):
            ecases.append(eras_case(223, e, x, True, 4))         # Q2: errors + erasures
    for x in (0, 3, 16):
        for _ in range(6):
            ecases.append(eras_case(223, 0, x, True, 5))         # Q3: e = 0, erasure-mode apply
    for e, x in ((32, 1), (30, 2), (16, 9)):
        for _ in range(6):
            ecases.append(eras_case(223, e, x, True, 6))         # beyond capacity with erasures
    for size in (40, 100):
        for _ in range(6):
            ecases.append(eras_case(size, 12, 3, True, 7))
    n = len(ecases)
    out["era_size"] = np.array([c["size"] for c in ecases], np.uint16)
    out["era_count"] = np.array([c["e"] for c in ecases], np.uint32)
    out["era_extra"] = np.array([c["x"] for c in ecases], np.uint16)
    out["era_kind"] = np.array([c["kind"] for c in ecases], np.uint8)
    out["era_slots"] = np.stack([c["slots"] for c in ecases]).astype(np.uint32)
    out["era_in"] = np.zeros((n, 255), np.uint8)
    out["era_out"] = np.zeros((n, 255), np.uint8)
    out["era_clean"] = np.zeros((n, 255), np.uint8)
    for i, c in enumerate(ecases):
        L = c["size"] + NR
        out["era_in"][i, :L] = c["inp"]
        out["era_out"][i, :L] = c["out"]
        out["era_clean"][i, :L] = c["clean"]
    out["era_ok"] = np.array([c["ok"] for c in ecases], np.uint8)
    out["era_cor"] = np.array([c["cor"] for c in ecases], np.uint32)
    eref.close()

    # ---- external syndromes (config "syndrome" pointer): all-A0 is a no-op
    # (tests/test_codec.c:78-121); also real syndromes of corrupted words.
    xs_in, xs_syn, xs_ok, xs_cor, xs_out = [], [], [], [], []
    for k in range(24):
        d = rng.integers(0, 256, 223, dtype=np.uint8)
        _, p = ref.encode(d)
        cw = np.concatenate([d, p])
        ne = 0 if k < 4 else int(rng.integers(1, 20))
        pos = rng.permutation(255)[:ne]
        cw[pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
        ref.decode(cw[:223], cw[223:])
        syn = np.full(NR, 255, np.uint16) if k < 4 else ref.last_syndrome()
        xr = Reference(ext_syn=syn)
        ok, n, od, op = xr.decode(cw[:223], cw[223:])
        xr.close()
        xs_in.append(cw), xs_syn.append(syn), xs_ok.append(ok), xs_cor.append(n)
        xs_out.append(np.concatenate([od, op]))
    out["xs_in"], out["xs_syn"] = np.stack(xs_in), np.stack(xs_syn)
    out["xs_ok"], out["xs_cor"], out["xs_out"] = np.array(xs_ok, np.uint8), np.array(xs_cor, np.uint32), np.stack(xs_out)

    # ---- invalid sizes (src/decode.c:418-429, :596-600)
    inv = []
    for size in (0, 224, 255):
        d = np.zeros(max(size, 1), np.uint8)
        ok, n, _, _ = ref.decode(d[:size] if size else d[:0], np.zeros(NR, np.uint8))
        inv.append((size, int(ok), n))
    out["invalid"] = np.array(inv, np.uint32)
    ref.close()

    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {os.path.getsize(OUT)} bytes; decode cases {len(cases)} "
          f"(miscorrections {sum(c['ok'] for c in misc)}), erasure cases {len(ecases)}")


if __name__ == "__main__":
    main()
