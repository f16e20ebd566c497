"""CPU checks of the algebra behind the split decode of codes with fewer
than 32 roots (api.cpp build_lfsr_rows / build_decode_tables with nr < 32,
rs_kernels.hip rsk_syndrome_reset_nr), against the oracle:

* the 32-byte LFSR with rows fb * g(x) x^(32 - nr) leaves the parity
  m(x) x^nr mod g(x) in its first nr bytes and zeros behind them;
* S_i of a received word equals E'(beta_i), E' = received parity + the parity
  of the received data (nr bytes, byte m the coefficient of x^(nr-1-m)),
  which is what the nibble tables compute (rows beta_i^(nr-1-m), zero rows
  for i >= nr and m >= nr);
* leading zero bytes leave the LFSR remainder unchanged (the block path of
  rs_lfsr_k feeds 16 nb - size of them).
"""
import numpy as np
import pytest

from oracle import Oracle

PARAMS = [(8, 0x11D, 1, 1, 16), (8, 0x187, 5, 1, 31), (8, 0x11D, 0, 1, 2), (8, 0x171, 1, 11, 10),
          (8, 0x11D, 1, 1, 32)]


def _gf(poly):
    exp = np.zeros(512, np.int64)
    log = np.zeros(256, np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= poly
    exp[255:510] = exp[:255]
    return exp, log


def _mul(exp, log, a, b):
    return 0 if a == 0 or b == 0 else int(exp[log[a] + log[b]])


def _generator(exp, log, fcr, prim, nr):
    """g(x) = prod (x + alpha^(prim (fcr + i))), coefficients low -> high"""
    g = [1]
    for i in range(nr):
        r = int(exp[(prim * (fcr + i)) % 255])
        ng = [0] * (len(g) + 1)
        for j, c in enumerate(g):
            ng[j + 1] ^= c
            ng[j] ^= _mul(exp, log, c, r)
        g = ng
    return g


def _lfsr32(exp, log, g, nr, msg):
    """the kernel's 32-byte register with rows fb * g_(nr-1-m) for m < nr, 0 behind"""
    reg = [0] * 32
    for d in msg:
        fb = int(d) ^ reg[0]
        reg = reg[1:] + [0]
        for m in range(nr):
            reg[m] ^= _mul(exp, log, fb, g[nr - 1 - m])
    return reg


@pytest.mark.parametrize("params", PARAMS)
def test_lfsr_with_shifted_generator(params):
    m, poly, fcr, prim, nr = params
    o = Oracle(*params)
    exp, log = _gf(poly)
    g = _generator(exp, log, fcr, prim, nr)
    rng = np.random.default_rng(nr)
    for size in (1, 17, 100, 255 - nr):
        data = rng.integers(0, 256, (8, size), dtype=np.uint8)
        want = o.encode_batch(data)
        for c in range(8):
            reg = _lfsr32(exp, log, g, nr, data[c])
            assert reg[:nr] == list(want[c]) and not any(reg[nr:]), (size, c)
            z = int(rng.integers(1, 16))  # leading zeros: the block path's padding
            assert _lfsr32(exp, log, g, nr, np.concatenate([np.zeros(z, np.uint8), data[c]])) == reg


@pytest.mark.parametrize("params", PARAMS)
def test_syndromes_from_eprime(params):
    m, poly, fcr, prim, nr = params
    o = Oracle(*params)
    exp, log = _gf(poly)
    rng = np.random.default_rng(100 + nr)
    size = 255 - nr
    data = rng.integers(0, 256, (20, size), dtype=np.uint8)
    par = o.encode_batch(data)
    for c in range(20):
        d, p = data[c].copy(), par[c].copy()
        ne = c % (nr // 2 + 3)
        cw = np.concatenate([d, p])
        pos = rng.permutation(size + nr)[:ne]
        cw[pos] ^= rng.integers(1, 256, ne).astype(np.uint8)
        d, p = cw[:size], cw[size:]
        eprime = p ^ o.encode_batch(d[None, :])[0]
        syn = []
        for i in range(nr):
            s = 0
            for mm in range(nr):  # the nibble tables' row for byte mm: beta_i^(nr - 1 - mm)
                s ^= _mul(exp, log, int(eprime[mm]), int(exp[((nr - 1 - mm) * prim * (fcr + i)) % 255]))
            syn.append(s)
        flag, want = o.syndrome(d, p)
        got = np.array([255 if v == 0 else log[v] for v in syn], np.uint16)
        assert (got == want).all() and flag == any(syn), c
