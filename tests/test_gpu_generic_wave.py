"""General-parameter kernels, one codeword per wave (rs_generic.hip
rsgw_encode_k / rsgw_decode_k) and one per lane (rsg_*), against the oracle
on every parameter set of the reference's own tests
(tests/golden/rs_params_golden.npz): 2..8-bit symbols, 2..200 roots, fcr 0..2000,
prim 1..37 -- including the sets whose exponents pass 2^16 (the syndromes'
Horner path) and those the reference itself fails at t errors.

Modes: encode (batch and single call), errors-only decode with 0 .. t + 2
errors, erasure decode with u8 slots (batch) and u32 slots (single call
through the erasure object, stale slots past the count included), external
syndromes (the row's own, random, all-zero and out-of-table values).
POPORON_AMD_GENERIC=wave|lane selects the kernel family (read at
poporon_create)."""
import os

import numpy as np
import pytest

import libpoporon_amd as P

pytestmark = pytest.mark.gpu

_PARAMS = [tuple(int(x) for x in p) for p in
           np.load(os.path.join(os.path.dirname(__file__), "golden", "rs_params_golden.npz"))["params"]]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _rows(rng, o, n, size, nn):
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)  # raw bytes: the codec masks to m bits
    return data, o.encode_batch(data)


@pytest.mark.parametrize("path", ["wave", "lane"])
@pytest.mark.parametrize("params", _PARAMS)
def test_generic_paths_vs_oracle(params, path, monkeypatch):
    from oracle import Oracle
    monkeypatch.setenv("POPORON_AMD_GENERIC", path)
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    assert h.supported
    nn = (1 << m) - 1
    k = nn - nr
    t = nr // 2
    rng = np.random.default_rng(sum(params) + (path == "lane"))
    n = 300 if nr < 100 else 120
    for size in sorted({k, max(1, k // 2), 1}):
        data, par = _rows(rng, o, n, size, nn)
        assert (h.encode_batch(data) == par).all(), size
        for c in range(0, n, 97):
            assert (h.encode(data[c]) == par[c]).all(), (size, c)
        # errors
        cw = np.concatenate([data, par], 1)
        for c in range(n):
            ne = min(c % (t + 3), size + nr)
            pos = rng.permutation(size + nr)[:ne]
            cw[c, pos] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
        ook, ocor, od, op = o.decode_batch(cw[:, :size], cw[:, size:])
        ok, cor, d, p = h.decode_batch(cw[:, :size], cw[:, size:])
        assert (ok == ook).all() and (cor == ocor).all(), size
        assert (d == od).all() and (p == op).all(), size
        for c in range(0, n, 61):
            sok, sn, sd, sp = h.decode(cw[c, :size], cw[c, size:])
            assert sok == bool(ook[c]) and sn == ocor[c] and (sd == od[c]).all() and (sp == op[c]).all(), (size, c)
        # erasures (+ errors): u8 slots, stale slots past the count
        cw = np.concatenate([data, par], 1)
        slots = np.zeros((n, nr), np.uint32)
        cnts = np.zeros(n, np.uint32)
        for c in range(n):
            e = int(rng.integers(0, nr + 1))
            extra = int(rng.integers(0, max(1, (nr - e) // 2 + 2)))
            perm = rng.permutation(size + nr)
            pos = perm[:min(e, size + nr)]
            slots[c, :len(pos)] = pos
            slots[c, len(pos):] = rng.integers(0, size + nr, nr - len(pos))
            cnts[c] = len(pos)
            cw[c, pos] ^= rng.integers(0, nn + 1, len(pos)).astype(np.uint8)
            ex = perm[len(pos):len(pos) + extra]
            cw[c, ex] ^= rng.integers(1, nn + 1, len(ex)).astype(np.uint8)
        ook, ocor, od, op = o.decode_batch(cw[:, :size], cw[:, size:], slots, cnts)
        ok, cor, d, p = h.decode_batch(cw[:, :size], cw[:, size:], slots.astype(np.uint8), cnts.astype(np.uint8))
        assert (ok == ook).all() and (cor == ocor).all(), ("era", size)
        assert (d == od).all() and (p == op).all(), ("era", size)
        er = P.Erasure(nr, nr)
        he = P.Poporon(m, poly, fcr, prim, nr, erasure=er)
        for c in range(0, n, 53):
            er.set(slots[c])  # the stale slots past the count stay in the object, as in the reference
            er.set(slots[c][:cnts[c]])
            sok, sn, sd, sp = he.decode(cw[c, :size], cw[c, size:])
            assert sok == bool(ook[c]) and sn == ocor[c] and (sd == od[c]).all() and (sp == op[c]).all(), c
        he.close()
    h.close()


@pytest.mark.parametrize("path", ["wave", "lane"])
@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 100), (8, 0x187, 5, 7, 48), (4, 0x13, 1, 2, 8),
                                    (8, 0x11D, 2000, 37, 32), (6, 0x43, 1, 1, 10)])
def test_generic_external_syndromes_vs_oracle(torch_cuda, params, path, monkeypatch):
    from oracle import Oracle
    torch = torch_cuda
    monkeypatch.setenv("POPORON_AMD_GENERIC", path)
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    nn = (1 << m) - 1
    k = nn - nr
    rng = np.random.default_rng(nr + 3)
    n = 300  # >= GW_GROUP_MIN: short codes on the grouped wave kernel (4 or 2 codewords per wave)
    data, par = _rows(rng, o, n, k, nn)
    cw = np.concatenate([data, par], 1)
    syn = np.zeros((n, nr), np.uint16)
    for c in range(n):
        ne = c % (nr // 2 + 2)
        pos = rng.permutation(nn)[:ne]
        cw[c, pos] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
        kind = c % 4
        if kind == 0:
            syn[c] = o.syndrome(cw[c, :k], cw[c, k:])[1]
        elif kind == 1:
            syn[c] = rng.integers(0, nn + 1, nr)
        elif kind == 2:
            syn[c] = nn
        else:
            syn[c] = o.syndrome(cw[c, :k], cw[c, k:])[1]
            syn[c, rng.integers(0, nr)] = nn + 1 + int(rng.integers(0, 300))
    dev = torch.from_numpy(cw.copy()).cuda()
    sy = torch.from_numpy(syn.astype(np.int16)).cuda()
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    cor = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    b = dev.data_ptr()
    h.decode_batch_syndrome_device(b, nn, b + k, nn, k, n, sy.data_ptr(), nr, ok.data_ptr(), cor.data_ptr(), s)
    torch.cuda.synchronize()
    got, gok, gcor = dev.cpu().numpy(), ok.cpu().numpy(), cor.cpu().numpy()
    for c in range(n):
        if (syn[c] > nn).any():  # out of the reference's tables: refused, untouched
            wok, wn, wd, wp = False, 0, cw[c, :k], cw[c, k:]
        else:
            wok, wn, wd, wp = o.decode(cw[c, :k], cw[c, k:], ext_syn=syn[c])
        assert gok[c] == wok and gcor[c] == wn, (c, c % 4)
        assert (got[c, :k] == wd).all() and (got[c, k:] == wp).all(), (c, c % 4)
    h.close()


@pytest.mark.parametrize("path", ["wave", "lane"])
@pytest.mark.parametrize("params", _PARAMS)
def test_generic_check_and_syndromes_vs_oracle(torch_cuda, params, path, monkeypatch):
    """poporon_check_batch_device / poporon_syndrome_batch_device on the
    general kernels (rsgw_check_k / rsg_check_k; the fewer-roots sets on the
    LFSR kernel): dirty flags and log-form syndromes equal the oracle's."""
    from oracle import Oracle
    torch = torch_cuda
    monkeypatch.setenv("POPORON_AMD_GENERIC", path)
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    nn = (1 << m) - 1
    rng = np.random.default_rng(nr * 5 + m)
    s = torch.cuda.current_stream().cuda_stream
    n = 200
    for size in sorted({nn - nr, max(1, (nn - nr) // 3)}):
        data, par = _rows(rng, o, n, size, nn)
        cw = np.concatenate([data, par], 1)
        for c in range(n):
            ne = c % 3
            cw[c, rng.permutation(size + nr)[:ne]] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
        dev = torch.from_numpy(cw).cuda()
        b, w = dev.data_ptr(), size + nr
        dirty = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        h.check_batch_device(b, w, b + size, w, size, n, dirty.data_ptr(), s)
        syn = torch.zeros((n, nr), dtype=torch.int16, device="cuda")
        nz = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        h.syndrome_batch_device(b, w, b + size, w, size, n, syn.data_ptr(), nr, nz.data_ptr(), s)
        torch.cuda.synchronize()
        got = syn.cpu().numpy().astype(np.uint16)
        gd, gn = dirty.cpu().numpy(), nz.cpu().numpy()
        for c in range(n):
            f, want = o.syndrome(cw[c, :size], cw[c, size:])
            assert bool(gd[c]) == f and bool(gn[c]) == f and (got[c] == want).all(), (size, c)
    h.close()


@pytest.mark.parametrize("path", ["wave", "lane"])
@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 100), (4, 0x13, 1, 2, 8), (8, 0x11D, 2000, 37, 32)])
def test_generic_single_call_edges_vs_oracle(params, path, monkeypatch):
    """Single calls on the general kernels at the branch edges: external
    syndromes (own, random, all nn, and a value past the field: refused with
    the bytes untouched), erasure counts 0 .. nr + 2 with stale slots (past nr
    on a dirty codeword: refused, Q5; on a clean one: success), shortened
    sizes 1 and k, against the oracle."""
    from oracle import Oracle
    monkeypatch.setenv("POPORON_AMD_GENERIC", path)
    m, poly, fcr, prim, nr = params
    nn = (1 << m) - 1
    k = nn - nr
    o = Oracle(*params)
    rng = np.random.default_rng(nr + m + 11)
    syn = np.zeros(nr, np.uint16)
    hx = P.Poporon(m, poly, fcr, prim, nr, syndrome=syn)
    er = P.Erasure(nr, nr + 4)
    he = P.Poporon(m, poly, fcr, prim, nr, erasure=er)
    for size in (k, 1):
        for c in range(24):
            data = rng.integers(0, nn + 1, size, dtype=np.uint8)
            par = o.encode(data)
            cw = np.concatenate([data, par])
            ne = c % (nr // 2 + 2)
            if c % 5 == 4:
                ne = 0  # clean
            pos = rng.permutation(size + nr)[:ne]
            cw[pos] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
            d, p = cw[:size], cw[size:]
            # external syndromes (the handle reads the array live)
            kind = c % 4
            if kind == 0:
                syn[:] = o.syndrome(d, p)[1]
            elif kind == 1:
                syn[:] = rng.integers(0, nn + 1, nr)
            elif kind == 2:
                syn[:] = nn
            else:
                syn[:] = o.syndrome(d, p)[1]
                syn[rng.integers(0, nr)] = nn + 1
            hx._syn[:] = syn
            got = hx.decode(d, p)
            if (syn > nn).any():
                want = (False, 0, d, p)
            else:
                want = o.decode(d, p, ext_syn=syn)
            assert got[0] == want[0] and got[1] == want[1], (size, c, kind)
            assert (got[2] == want[2]).all() and (got[3] == want[3]).all(), (size, c, kind)
            # erasures: count 0 .. nr + 2, stale slots from the previous fill
            e = c % (nr + 3)
            slots = rng.integers(0, size + nr, nr + 4).astype(np.uint32)
            er.set(slots)
            er.set(slots[:e])
            got = he.decode(d, p)
            if e > nr:  # Q5 (undefined in the reference): refused for a dirty codeword, success for a clean one
                want = (not o.syndrome(d, p)[0], 0, d, p)
            else:  # count e, the row's nr slots with the stale ones past e (Q2)
                wok, wcor, wd, wp = o.decode_batch(d[None, :], p[None, :], slots[None, :nr],
                                                   np.array([e], np.uint32))
                want = (bool(wok[0]), int(wcor[0]), wd[0], wp[0])
            assert got[0] == want[0] and got[1] == want[1], (size, c, e)
            assert (got[2] == want[2]).all() and (got[3] == want[3]).all(), (size, c, e)
    hx.close()
    he.close()


@pytest.mark.parametrize("params", [(4, 0x13, 1, 2, 8), (8, 0x11D, 1, 1, 100), (7, 0x89, 1, 1, 20)])
def test_generic_single_call_server_vs_oracle(params):
    """The general-parameter single-call server (rsgw_serve_k): calls spaced
    around its 1 ms idle limit (it leaves and is launched again), device
    batches and synchronisations in between, a second general handle and an
    RS(255,223) handle (rs_serve_k) serving at the same time, the per-call
    launch path (kernel timing on) interleaved, shortened sizes (the staged
    encode rows change with the size), and a close that stops a live server
    -- every result equal to the oracle's."""
    import time

    import torch
    from oracle import Oracle
    m, poly, fcr, prim, nr = params
    nn = (1 << m) - 1
    k = nn - nr
    o, od = Oracle(*params), Oracle()
    h, h2, hd = P.Poporon(*params), P.Poporon(*params), P.Poporon.default()
    rng = np.random.default_rng(nr * 3 + m)
    for c in range(40):
        if c % 3 == 0:
            time.sleep([0.0, 0.0009, 0.0011, 0.003][(c // 3) % 4])
        if c % 8 == 5:
            torch.cuda.synchronize()
        size = k if c % 4 else int(rng.integers(1, k + 1))
        data = rng.integers(0, nn + 1, size, dtype=np.uint8)
        want = o.encode(data)
        hh = h if c % 2 else h2
        timing = c % 5 == 3
        hh.timing(timing)  # kernel timing on: one launch per call instead of the server
        if c % 8 == 6:
            bd = np.tile(data, (3, 1))
            okb, corb, db, pb = hh.decode_batch(bd, np.tile(want, (3, 1)))
            assert okb.all() and (db == bd).all()
        assert (hh.encode(data) == want).all(), c
        cw = np.concatenate([data, want])
        ne = int(rng.integers(0, nr // 2 + 1))
        cw[rng.permutation(size + nr)[:ne]] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
        got = hh.decode(cw[:size], cw[size:])
        wok, wn, wd, wp = o.decode(cw[:size], cw[size:])
        assert got[0] == wok and got[1] == wn and (got[2] == wd).all() and (got[3] == wp).all(), c
        hh.timing(False)
        md = rng.integers(0, 256, 223, dtype=np.uint8)
        assert (hd.encode(md) == od.encode(md)).all(), c
    h.close()  # asks its live server to leave
    data = rng.integers(0, nn + 1, k, dtype=np.uint8)
    assert (h2.encode(data) == o.encode(data)).all()
    h2.close()
    hd.close()


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 100), (4, 0x13, 1, 2, 8), (7, 0x89, 1, 1, 20),
                                    (6, 0x43, 1, 1, 10), (5, 0x25, 3, 1, 6), (2, 0x7, 1, 1, 2)])
def test_generic_large_batch_round_trip(torch_cuda, params):
    """Large device batches on the default routing (decode: 64 lanes per
    codeword for 255-symbol codes, two codewords per pass; 32 / 16 / 8 lanes
    for codes of up to 127 / 63 / 31 symbols; one codeword per lane for
    3-symbol codes; encode per lane below 255 symbols): 2^18 rows
    encoded, t random errors each, decoded -- every row back to the encoded
    one with ok = 1 and corrected_num = t (a size-independent property), and
    every 1024th row equal to the oracle's encode and decode."""
    from oracle import Oracle
    torch = torch_cuda
    m, poly, fcr, prim, nr = params
    nn = (1 << m) - 1
    k, t = nn - nr, nr // 2
    n = 1 << 18
    o, h = Oracle(*params), P.Poporon(*params)
    rng = np.random.default_rng(nn + nr)
    data = rng.integers(0, nn + 1, (n, k), dtype=np.uint8)
    rows = torch.zeros((n, nn), dtype=torch.uint8, device="cuda")
    rows[:, :k] = torch.from_numpy(data).cuda()
    s = torch.cuda.current_stream().cuda_stream
    b = rows.data_ptr()
    h.encode_batch_device(b, nn, b + k, nn, k, n, s)
    torch.cuda.synchronize()
    clean = rows.cpu().numpy()
    idx = np.arange(0, n, 1024)
    assert (clean[idx, k:] == o.encode_batch(data[idx])).all()
    pos = np.argsort(rng.random((n, nn)), axis=1)[:, :t]
    bad = clean.copy()
    np.bitwise_xor.at(bad, (np.arange(n)[:, None], pos), rng.integers(1, nn + 1, (n, t), dtype=np.uint8))
    rows.copy_(torch.from_numpy(bad).cuda())
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    h.decode_batch_device(b, nn, b + k, nn, k, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    torch.cuda.synchronize()
    got = rows.cpu().numpy()
    assert bool((ok == 1).all()) and bool((cor == t).all())
    assert (got == clean).all()
    ook, ocor, od, op = o.decode_batch(bad[idx, :k], bad[idx, k:])
    assert (ook == 1).all() and (ocor == t).all() and (od == clean[idx, :k]).all() and (op == clean[idx, k:]).all()
    h.close()


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 100), (8, 0x187, 5, 7, 48), (8, 0x11D, 2000, 37, 32)])
def test_generic_pair_batches_vs_oracle(torch_cuda, params):
    """Batches large enough that each wave of rsgw_decode_k<., 64> takes two
    codewords per pass (gw_decode_pair: the first's syndromes kept aside,
    both Berlekamp-Massey runs interleaved, B finished before A), with every
    case mixed in: clean rows, 1..t errors, t+1..t+3 (the reference's
    failures and miscorrections) -- every row's bytes, ok and corrected_num
    against the oracle."""
    from oracle import Oracle
    torch = torch_cuda
    m, poly, fcr, prim, nr = params
    nn = (1 << m) - 1
    k, t = nn - nr, nr // 2
    n = 20000  # > the 8,192 waves of a capped grid: passes pair codewords e and e + 8192
    o, h = Oracle(*params), P.Poporon(*params)
    rng = np.random.default_rng(nr * 7 + fcr)
    data = rng.integers(0, nn + 1, (n, k), dtype=np.uint8)
    cw = np.concatenate([data, o.encode_batch(data)], 1)
    ne = rng.integers(0, t + 4, n)
    ne[rng.random(n) < 0.2] = 0  # clean rows beside dirty ones in the same pass
    for c in range(n):
        p = rng.permutation(nn)[:ne[c]]
        cw[c, p] ^= rng.integers(1, nn + 1, ne[c]).astype(np.uint8)
    rows = torch.from_numpy(cw).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    b = rows.data_ptr()
    h.decode_batch_device(b, nn, b + k, nn, k, n, ok.data_ptr(), cor.data_ptr(),
                          stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = rows.cpu().numpy()
    ook, ocor, od, op = o.decode_batch(cw[:, :k], cw[:, k:])
    assert (ok.cpu().numpy() == ook).all() and (cor.cpu().numpy() == ocor).all()
    assert (got[:, :k] == od).all() and (got[:, k:] == op).all()
    h.close()
