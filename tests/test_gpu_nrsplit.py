"""Byte-symbol codes with 2 <= num_roots < 32 on the split decode kernels
(api.cpp params_nrsplit / launch_split with npar = num_roots): syndromes from
the LFSR kernel with g(x) x^(32 - nr) (rsk_syndrome_reset_nr), nr BM
iterations with the fast path bounded by 2L <= nr (rs_bm_k<true>), the
unchanged Chien and Forney kernels, the block apply over size + nr bytes and
the general-parameter kernel over the hand-off list (rsg_decode_list).

Every result -- bytes, ok, corrected_num -- is compared with the oracle
(oracle/rs_oracle.c, pinned to the compiled reference by
tests/test_oracle_golden.py), over error counts 0 .. t + 3 (past the
capability too, so the list and the failure paths run), shortened sizes,
the wire layout (block apply) and strided rows (byte apply).  The kernel
timers prove the split kernels ran."""
import numpy as np
import pytest

import libpoporon_amd as P

pytestmark = pytest.mark.gpu

# (symbol_size, poly, fcr, prim, num_roots), split path expected: RS(255,239),
# t = 1, odd nr with fcr 5, nr 8 with fcr 3, prim 11 / 7 over other field
# polynomials; and two sets outside the fast path's exponent bound
# ((fcr + nr - 1) prim 254 >= 32768: RsCorrParams.vfast), which stay on the
# general kernel with the same results
PARAMS = [((8, 0x11D, 1, 1, 16), True), ((8, 0x11D, 0, 1, 2), True), ((8, 0x187, 5, 1, 31), True),
          ((8, 0x11D, 3, 1, 8), True), ((8, 0x171, 1, 11, 10), True), ((8, 0x187, 1, 7, 16), True),
          ((8, 0x187, 5, 7, 31), False), ((8, 0x171, 1, 11, 20), False)]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _channel(rng, data, par, nr, nmax):
    """codewords with 0 .. nmax errors at random positions (data and parity)"""
    n, k = data.shape
    cw = np.concatenate([data, par], 1)
    for c in range(n):
        ne = min(c % (nmax + 1), k + nr)
        pos = rng.permutation(k + nr)[:ne]
        cw[c, pos] ^= rng.integers(1, 256, ne).astype(np.uint8)
    return cw


def _bm_launches(h):
    return h.timing_read(P.KERNEL_BM)[1]


@pytest.mark.parametrize("params,split", PARAMS)
def test_nrsplit_vs_oracle(torch_cuda, params, split, monkeypatch):
    """POPORON_AMD_DECODE_PATH=split sends every errors-only batch to the
    split kernels: host batches and device batches (wire rows and strided
    rows) at full length and shortened, bit-exact against the oracle."""
    from oracle import Oracle
    torch = torch_cuda
    monkeypatch.setenv("POPORON_AMD_DECODE_PATH", "split")
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    assert h.supported
    t = nr // 2
    rng = np.random.default_rng(nr * 7919 + prim)
    s = torch.cuda.current_stream().cuda_stream
    for size in (255 - nr, (255 - nr) // 3, 1):
        n = 3000
        data = rng.integers(0, 256, (n, size), dtype=np.uint8)
        par = o.encode_batch(data)
        cw = _channel(rng, data, par, nr, t + 3)
        ook, ocor, od, op = o.decode_batch(cw[:, :size], cw[:, size:])
        assert (ook[(np.arange(n) % (t + 4)) <= t] == 1).all()  # within t: all corrected
        # host batch
        h.timing(True)
        ok, cor, d, p = h.decode_batch(cw[:, :size], cw[:, size:])
        assert (_bm_launches(h) > 0) == split, "split kernels ran" if not split else "split kernels did not run"
        h.timing(False)
        assert (ok == ook).all() and (cor == ocor).all(), size
        assert (d == od).all() and (p == op).all(), size
        # device batches: wire rows (size + nr bytes back to back) and strided rows
        for extra, off in ((0, 0), (5, 3)):
            w = size + nr + extra
            buf = np.zeros(n * w + off + 64, np.uint8)
            rows = buf[off:off + n * w].reshape(n, w)
            rows[:, :size + nr] = cw
            dev = torch.from_numpy(buf).cuda()
            okd = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
            cord = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
            b = dev.data_ptr() + off
            h.decode_batch_device(b, w, b + size, w, size, n, okd.data_ptr(), cord.data_ptr(), stream=s)
            torch.cuda.synchronize()
            got = dev.cpu().numpy()
            grows = got[off:off + n * w].reshape(n, w)
            assert (okd.cpu().numpy() == ook).all() and (cord.cpu().numpy() == ocor).all(), (size, extra)
            assert (grows[:, :size] == od).all() and (grows[:, size:size + nr] == op).all(), (size, extra)
            mask = np.ones(got.size, bool)  # nothing outside the codewords moved
            mask[off:off + n * w].reshape(n, w)[:, :size + nr] = False
            assert (got[mask] == buf[mask]).all(), (size, extra)


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 16), (8, 0x187, 5, 1, 31)])
def test_nrsplit_default_routing_large(torch_cuda, params, monkeypatch):
    """Without the override every errors-only batch takes the split kernels:
    40,000 wire rows with 0 .. t errors all corrected, a sample equal to the
    oracle, the rest checked by the round trip (bytes back to the encoded
    rows); POPORON_AMD_DECODE_PATH=single keeps a handle on the general
    kernel, with the same results; single calls agree with the oracle."""
    from oracle import Oracle
    torch = torch_cuda
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    t = nr // 2
    k = 255 - nr
    n = 40000
    rng = np.random.default_rng(nr)
    data = rng.integers(0, 256, (n, k), dtype=np.uint8)
    clean = np.concatenate([data, h.encode_batch(data)], 1)
    assert (clean[::97, k:] == o.encode_batch(data[::97])).all()
    cw = _channel(rng, data, clean[:, k:], nr, t)
    s = torch.cuda.current_stream().cuda_stream
    dev = torch.from_numpy(cw).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    h.timing(True)
    b = dev.data_ptr()
    h.decode_batch_device(b, 255, b + k, 255, k, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert _bm_launches(h) == 1
    h.timing(False)
    want_cor = np.array([((clean[c] != cw[c]).sum()) for c in range(n)], np.uint8)
    assert bool((ok == 1).all())
    assert (cor.cpu().numpy() == want_cor).all()
    assert (dev.cpu().numpy() == clean).all()
    ook, ocor, od, op = o.decode_batch(cw[::13, :k], cw[::13, k:])
    assert (ook == 1).all() and (ocor == want_cor[::13]).all()
    # a small batch: the split kernels too; forced onto the general kernel: same results
    monkeypatch.setenv("POPORON_AMD_DECODE_PATH", "single")
    hg = P.Poporon(*params)
    monkeypatch.delenv("POPORON_AMD_DECODE_PATH")
    for hh, launches in ((h, 1), (hg, 0)):
        hh.timing(True)
        small = torch.from_numpy(cw[:5000]).cuda()
        ok2 = torch.zeros(5000, dtype=torch.uint8, device="cuda")
        hh.decode_batch_device(small.data_ptr(), 255, small.data_ptr() + k, 255, k, 5000, ok2.data_ptr(), stream=s)
        torch.cuda.synchronize()
        assert _bm_launches(hh) == launches
        hh.timing(False)
        assert bool((ok2 == 1).all()) and (small.cpu().numpy() == clean[:5000]).all()
    # single calls (poporon_decode): the split kernels on one codeword
    for c in range(0, 64):
        ok1, n1, d1, p1 = h.decode(cw[c, :k], cw[c, k:])
        assert ok1 and n1 == want_cor[c] and (np.concatenate([d1, p1]) == clean[c]).all(), c


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 32), (8, 0x11D, 1, 1, 16), (8, 0x187, 5, 1, 31), (8, 0x11D, 0, 1, 2)])
def test_every_size_vs_oracle(torch_cuda, params, monkeypatch):
    """Every message size 1 .. 255 - nr through the batch encode and the
    split decode (POPORON_AMD_DECODE_PATH=split), rows at an odd offset and
    stride: the LFSR kernel's block path (16 <= size <= 256 but not the full
    RS(255,223): 16-byte blocks behind 16 nb - size leading zeros, every
    z = 0..15) and its dword path (size < 16) against the oracle."""
    from oracle import Oracle
    torch = torch_cuda
    monkeypatch.setenv("POPORON_AMD_DECODE_PATH", "split")
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    t = nr // 2
    rng = np.random.default_rng(nr + 4242)
    s = torch.cuda.current_stream().cuda_stream
    n, off = 96, 3
    for size in range(1, 256 - nr):
        w = size + nr + 1
        data = rng.integers(0, 256, (n, size), dtype=np.uint8)
        want = o.encode_batch(data)
        buf = np.zeros(n * w + off + 64, np.uint8)
        rows = buf[off:off + n * w].reshape(n, w)
        rows[:, :size] = data
        dev = torch.from_numpy(buf).cuda()
        b = dev.data_ptr() + off
        h.encode_batch_device(b, w, b + size, w, size, n, s)
        torch.cuda.synchronize()
        got = dev.cpu().numpy()[off:off + n * w].reshape(n, w)
        assert (got[:, size:size + nr] == want).all(), size
        for c in range(0, n, 32):  # single calls (rs_enc1_k with the code's encq rows)
            assert (h.encode(data[c]) == want[c]).all(), (size, c)
        cw = _channel(rng, data, want, nr, t)
        rows[:, :size + nr] = cw
        dev = torch.from_numpy(buf).cuda()
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
        b = dev.data_ptr() + off
        h.decode_batch_device(b, w, b + size, w, size, n, ok.data_ptr(), cor.data_ptr(), stream=s)
        torch.cuda.synchronize()
        ook, ocor, od, op = o.decode_batch(cw[:, :size], cw[:, size:])
        got = dev.cpu().numpy()[off:off + n * w].reshape(n, w)
        assert (ok.cpu().numpy() == ook).all() and (cor.cpu().numpy() == ocor).all(), size
        assert (got[:, :size] == od).all() and (got[:, size:size + nr] == op).all(), size


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 16), (8, 0x187, 5, 1, 31), (8, 0x11D, 3, 1, 8),
                                    (8, 0x171, 1, 11, 10), (8, 0x11D, 0, 1, 2)])
@pytest.mark.parametrize("split", [True, False])
def test_nrsplit_erasures_vs_oracle(torch_cuda, params, split, monkeypatch):
    """Erasure batches of a code with fewer than 32 roots (u8 slots) on the
    errata kernels with npar = nr (rsk_ebm_nr, rsk_chien32, rsk_forney32_nr,
    the list on rsg_decode_k in erasure mode, rsk_apply_era_nr), or, with
    POPORON_AMD_DECODE_PATH=single, on the general kernel: bytes, ok and
    corrected_num equal the oracle's over erasure counts 0 .. nr + 2 (past
    nr: refused when dirty, quirk Q5), errors besides (within and past the
    capability), unsorted and repeated slots (Q1), slots read past the count
    (Q2), slots past the codeword, shortened sizes, rows of slots at a stride
    of roundup(nr, 4) (the errata path) and nr + 1 (the general kernel)."""
    from oracle import Oracle
    torch = torch_cuda
    monkeypatch.setenv("POPORON_AMD_DECODE_PATH", "split" if split else "single")
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    rng = np.random.default_rng(nr * 31 + fcr)
    s = torch.cuda.current_stream().cuda_stream
    for size in (255 - nr, (255 - nr) // 2):
        n = 2000
        data = rng.integers(0, 256, (n, size), dtype=np.uint8)
        cw = np.concatenate([data, o.encode_batch(data)], 1)
        slots = np.zeros((n, nr), np.uint8)
        cnts = np.zeros(n, np.uint8)
        for c in range(n):
            e = c % (nr + 3)
            pos = rng.permutation(size + nr)[:min(e, size + nr)]
            if c % 3:
                pos = np.sort(pos)
            if c % 7 == 0 and len(pos) > 1:
                pos[-1] = pos[0]  # a repeated slot
            if c % 11 == 0 and len(pos):
                pos[-1] = min(255, size + nr + int(rng.integers(0, 8)))  # past the codeword
            k = min(len(pos), nr)
            slots[c, :k] = pos[:k]
            slots[c, k:] = rng.integers(0, size, nr - k)  # stale entries past the count
            cnts[c] = e
            inside = pos[pos < size + nr]
            cw[c, inside] ^= rng.integers(1, 256, len(inside)).astype(np.uint8)
            room = max(0, (nr - min(e, nr)) // 2 + (1 if c % 5 == 0 else 0))  # one past the capability at times
            free = np.setdiff1d(np.arange(size + nr), pos)
            pe = rng.permutation(free)[:room]
            cw[c, pe] ^= rng.integers(1, 256, len(pe)).astype(np.uint8)
        ook, ocor, od, op = o.decode_batch(cw[:, :size], cw[:, size:], slots.astype(np.uint32), cnts.astype(np.uint32))
        for ps in ((nr + 3) // 4 * 4, nr + 1):
            sl = np.zeros((n, ps), np.uint8)
            sl[:, :nr] = slots
            dev = torch.from_numpy(np.ascontiguousarray(cw)).cuda()
            dsl = torch.from_numpy(sl).cuda()
            dcn = torch.from_numpy(cnts).cuda()
            ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
            cor = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
            b = dev.data_ptr()
            h.timing(True)
            h.decode_batch_device(b, size + nr, b + size, size + nr, size, n, ok.data_ptr(), cor.data_ptr(),
                                  d_positions=dsl.data_ptr(), positions_stride=ps, d_counts=dcn.data_ptr(), stream=s)
            torch.cuda.synchronize()
            errata = _bm_launches(h) > 0
            h.timing(False)
            assert errata == (split and ps % 4 == 0), (size, ps)
            got = dev.cpu().numpy()
            assert (ok.cpu().numpy() == ook).all() and (cor.cpu().numpy() == ocor).all(), (size, ps)
            assert (got[:, :size] == od).all() and (got[:, size:] == op).all(), (size, ps)


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 16), (8, 0x187, 5, 1, 31)])
def test_nrsplit_single_call_erasures_vs_oracle(torch_cuda, params):
    """poporon_decode with an erasure object on a code with fewer than 32
    roots: slots below 255 go to the errata kernels as u8 slots, a slot of
    255 or more keeps the general kernel's u32 path; either way the bytes,
    the result and corrected_num equal the oracle's (stale slots past the
    count included, quirk Q2; counts past nr, Q5)."""
    from oracle import Oracle
    m, poly, fcr, prim, nr = params
    o = Oracle(*params)
    er = P.Erasure(nr, nr)
    h = P.Poporon(*params, erasure=er)
    rng = np.random.default_rng(nr + 99)
    k = 255 - nr
    for c in range(120):
        data = rng.integers(0, 256, (1, k), dtype=np.uint8)
        cw = np.concatenate([data, o.encode_batch(data)], 1)[0]
        e = c % (nr + 2)
        pos = np.sort(rng.permutation(k)[:min(e, k)])
        slots = np.zeros(nr, np.uint32)
        slots[:min(e, nr)] = pos[:nr]
        slots[min(e, nr):] = rng.integers(0, k, nr - min(e, nr))
        if c % 9 == 0:
            slots[-1] = 300  # a slot past a byte: the u32 path
        cw[pos] ^= rng.integers(1, 256, len(pos)).astype(np.uint8)
        ne = max(0, (nr - e) // 2)
        free = np.setdiff1d(np.arange(255), pos)
        pe = rng.permutation(free)[:ne]
        cw[pe] ^= rng.integers(1, 256, ne).astype(np.uint8)
        er.set(slots)
        er.set(slots[:e] if e <= nr else np.concatenate([slots, rng.integers(0, k, e - nr).astype(np.uint32)]))
        ok, n, d, p = h.decode(cw[:k], cw[k:])
        cnt = np.array([e], np.uint32)
        ook, ocor, od, op = o.decode_batch(cw[None, :k], cw[None, k:], slots[None, :].astype(np.uint32), cnt)
        assert ok == bool(ook[0]) and n == ocor[0], c
        assert (d == od[0]).all() and (p == op[0]).all(), c


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 16), (8, 0x187, 5, 1, 31), (8, 0x11D, 0, 1, 2)])
def test_nrsplit_check_and_syndromes_vs_oracle(torch_cuda, params):
    """poporon_check_batch_device and poporon_syndrome_batch_device of a code
    with fewer than 32 roots on the LFSR kernel (rsk_check_nr,
    rsk_syndrome_reset_nr + rsk_syn_log_nr): the dirty flags and the npar
    log-form syndromes (rows of exactly nr entries, the next row right
    behind) equal the oracle's, full-length and shortened, clean and dirty."""
    from oracle import Oracle
    torch = torch_cuda
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    rng = np.random.default_rng(nr + 7)
    s = torch.cuda.current_stream().cuda_stream
    for size in (255 - nr, 40):
        n = 3000
        data = rng.integers(0, 256, (n, size), dtype=np.uint8)
        cw = np.concatenate([data, o.encode_batch(data)], 1)
        for c in range(n):
            ne = c % 4
            cw[c, rng.permutation(size + nr)[:ne]] ^= rng.integers(1, 256, ne).astype(np.uint8)
        dev = torch.from_numpy(cw).cuda()
        b, w = dev.data_ptr(), size + nr
        dirty = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        h.check_batch_device(b, w, b + size, w, size, n, dirty.data_ptr(), s)
        syn = torch.zeros((n, nr), dtype=torch.int16, device="cuda")
        nz = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        h.syndrome_batch_device(b, w, b + size, w, size, n, syn.data_ptr(), nr, nz.data_ptr(), s)
        torch.cuda.synchronize()
        got_syn = syn.cpu().numpy().astype(np.uint16)
        for c in range(n):
            f, want = o.syndrome(cw[c, :size], cw[c, size:])
            assert bool(dirty[c]) == f and bool(nz[c]) == f and (got_syn[c] == want).all(), (size, c)


@pytest.mark.parametrize("params,path", [((8, 0x11D, 1, 1, 32), "split"), ((8, 0x11D, 1, 1, 32), None),
                                         ((8, 0x11D, 1, 1, 16), None), ((8, 0x187, 5, 1, 31), None),
                                         ((8, 0x11D, 0, 1, 2), None), ((8, 0x171, 1, 11, 10), "split")])
def test_external_syndrome_batches_vs_oracle(torch_cuda, params, path, monkeypatch):
    """poporon_decode_batch_syndrome_device on the split kernels
    (rsk_ext_syn converts the log-form syndromes; a value > 255 refuses its
    codeword through the list): the received word's own syndromes, random
    syndromes, all-255 rows (clean) and rows holding a value > 255, against
    the oracle's decode with the same external syndromes (src/decode.c:446-464).
    RS(255,223) with the override and at 20,000 codewords (the default's split
    threshold is 16,384); fewer-roots codes at every count."""
    from oracle import Oracle
    torch = torch_cuda
    if path:
        monkeypatch.setenv("POPORON_AMD_DECODE_PATH", path)
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    rng = np.random.default_rng(nr * 31 + prim)
    s = torch.cuda.current_stream().cuda_stream
    n = 20000 if (nr == 32 and path is None) else 3000
    nchk = 3000  # rows checked against the oracle; the rest by the round trip
    for size in (255 - nr, 60):
        data = rng.integers(0, 256, (n, size), dtype=np.uint8)
        clean = np.concatenate([data, o.encode_batch(data)], 1)
        cw = _channel(rng, data, clean[:, size:].copy(), nr, nr // 2)
        syn = np.zeros((n, nr), np.uint16)
        for c in range(n):
            kind = c % 5 if c < nchk else 0
            if kind in (0, 1):
                syn[c] = o.syndrome(cw[c, :size], cw[c, size:])[1]
            elif kind == 2:
                syn[c] = rng.integers(0, 256, nr)
            elif kind == 3:
                syn[c] = 255
            else:
                syn[c] = o.syndrome(cw[c, :size], cw[c, size:])[1]
                syn[c, rng.integers(0, nr)] = int(rng.integers(256, 65536))
        dev = torch.from_numpy(cw).cuda()
        sy = torch.from_numpy(syn.astype(np.int16)).cuda()
        ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        cor = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        b, w = dev.data_ptr(), size + nr
        h.timing(True)
        h.decode_batch_syndrome_device(b, w, b + size, w, size, n, sy.data_ptr(), nr, ok.data_ptr(), cor.data_ptr(), s)
        torch.cuda.synchronize()
        assert _bm_launches(h) > 0, "split kernels did not run"
        h.timing(False)
        got, gok, gcor = dev.cpu().numpy(), ok.cpu().numpy(), cor.cpu().numpy()
        for c in range(nchk):
            if (syn[c] > 255).any():  # out of the reference's tables (no defined result): refused, untouched
                wok, wn, wd, wp = False, 0, cw[c, :size], cw[c, size:]
            else:
                wok, wn, wd, wp = o.decode(cw[c, :size], cw[c, size:], ext_syn=syn[c])
            assert gok[c] == wok and gcor[c] == wn, (size, c, c % 5)
            assert (got[c, :size] == wd).all() and (got[c, size:] == wp).all(), (size, c, c % 5)
        assert (gok[nchk:] == 1).all() and (got[nchk:] == clean[nchk:]).all()
