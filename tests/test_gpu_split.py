"""GPU parity of the split error-mode decode (rs_fast.hip: rs_bm_k, rs_chien_k,
rs_forney_k, and the general kernel over the codewords they hand on).

POPORON_AMD_DECODE_PATH (read at poporon_create) forces the split kernels or
the single correction kernel whatever the batch size, so both paths meet the
same inputs; the expected values come from the golden fixtures (the compiled
reference, tools/gen_golden.py) or the pinned CPU oracle.  Everything is
compared bit-exactly: bytes, the bool result and corrected_num.
"""
import numpy as np
import pytest

import libpoporon_amd as P

pytestmark = pytest.mark.gpu

NR = 32
PATHS = ["split", "single", "wave"]


def _handle(monkeypatch, path, params=(8, 0x11D, 1, 1, 32)):
    if P.device_count() == 0:
        pytest.fail("no HIP device: GPU tests must run on the MI355X box")
    monkeypatch.setenv("POPORON_AMD_DECODE_PATH", path)
    h = P.Poporon(*params)
    assert h.supported
    return h


def _same(got, want):
    ok, cor, d, p = got
    ook, ocor, od, op = want
    assert (ok == ook).all(), np.nonzero(ok != ook)[0][:8]
    assert (cor == ocor).all(), np.nonzero(cor != ocor)[0][:8]
    assert (d == od).all() and (p == op).all()


def test_split_golden(monkeypatch, golden):
    h = _handle(monkeypatch, "split")
    sizes = golden["dec_size"]
    for s in np.unique(sizes):
        sel = np.nonzero(sizes == s)[0]
        s = int(s)
        ok, cor, d, p = h.decode_batch(golden["dec_in"][sel, :s], golden["dec_in"][sel, s:s + NR])
        assert (ok == golden["dec_ok"][sel]).all(), s
        assert (cor == golden["dec_cor"][sel]).all(), s
        assert (np.concatenate([d, p], 1) == golden["dec_out"][sel, :s + NR]).all(), s


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("size", [223, 200, 17, 1])
def test_split_random_vs_oracle(monkeypatch, oracle_default, path, size):
    """0..20 random errors (clean, correctable and beyond-capacity codewords
    side by side in every wave), shortened codes included."""
    h = _handle(monkeypatch, path)
    rng = np.random.default_rng(1000 + size)
    n = 12000
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    L = size + NR
    ne = rng.integers(0, min(21, L + 1), n)
    for c in range(n):
        pos = rng.permutation(L)[: ne[c]]
        cw[c, pos] ^= rng.integers(1, 256, ne[c], dtype=np.uint8)
    got = h.decode_batch(cw[:, :size], cw[:, size:])
    _same(got, oracle_default.decode_batch(cw[:, :size], cw[:, size:]))


@pytest.mark.parametrize("path", PATHS)
def test_split_beyond_capacity_vs_oracle(monkeypatch, oracle_default, path):
    """14..32 errors: codewords the split kernels hand to the general kernel
    (L > 16, deg != L, a locator past x^16) and the miscorrections the
    reference makes, bit for bit."""
    h = _handle(monkeypatch, path)
    rng = np.random.default_rng(77)
    n = 30000
    data = rng.integers(0, 256, (n, 223), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    for c in range(n):
        ne = int(rng.integers(14, 33))
        pos = rng.permutation(255)[:ne]
        cw[c, pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
    got = h.decode_batch(cw[:, :223], cw[:, 223:])
    want = oracle_default.decode_batch(cw[:, :223], cw[:, 223:])
    assert want[0].sum() > n // 10 and (~want[0].astype(bool)).sum() > n // 10
    _same(got, want)


def test_split_constructed_miscorrections(monkeypatch, golden, oracle_default):
    """The golden file's constructed miscorrections (words next to another
    codeword) and beyond-capacity failures, repeated to fill whole waves."""
    h = _handle(monkeypatch, "split")
    sel = np.nonzero(golden["dec_size"] == 223)[0]
    inp = np.tile(golden["dec_in"][sel], (8, 1))
    got = h.decode_batch(inp[:, :223], inp[:, 223:NR + 223])
    _same(got, oracle_default.decode_batch(inp[:, :223], inp[:, 223:NR + 223]))


@pytest.mark.parametrize("params", [(8, 0x11D, 0, 1, 32), (8, 0x11D, 2, 1, 32), (8, 0x11D, 1, 2, 32),
                                    (8, 0x187, 1, 1, 32), (8, 0x11D, 5, 7, 32)])
def test_split_other_parameters_vs_oracle(monkeypatch, params):
    from oracle import Oracle
    o = Oracle(*params)
    h = _handle(monkeypatch, "split", params)
    rng = np.random.default_rng(sum(params))
    n = 9000
    data = rng.integers(0, 256, (n, 223), dtype=np.uint8)
    par = h.encode_batch(data)
    assert (par == o.encode_batch(data)).all()
    cw = np.concatenate([data, par], 1)
    for c in range(n):
        ne = int(rng.integers(0, 23))
        pos = rng.permutation(255)[:ne]
        cw[c, pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
    _same(h.decode_batch(cw[:, :223], cw[:, 223:]), o.decode_batch(cw[:, :223], cw[:, 223:]))


@pytest.mark.parametrize("offset,stride", [(1, 257), (3, 256), (0, 255)])
def test_split_device_strides(monkeypatch, oracle_default, offset, stride):
    import torch
    h = _handle(monkeypatch, "split")
    rng = np.random.default_rng(stride + offset)
    n = 20000
    data = rng.integers(0, 256, (n, 223), dtype=np.uint8)
    cw = np.concatenate([data, oracle_default.encode_batch(data)], 1)
    for c in range(n):
        ne = int(rng.integers(0, 19))
        pos = rng.permutation(255)[:ne]
        cw[c, pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
    buf = np.zeros(offset + n * stride, np.uint8)
    rows = buf[offset:].reshape(n, stride)
    rows[:, :255] = cw
    d = torch.from_numpy(buf).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    base = d.data_ptr() + offset
    s = torch.cuda.current_stream().cuda_stream
    h.decode_batch_device(base, stride, base + 223, stride, 223, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    torch.cuda.synchronize()
    out = d.cpu().numpy()[offset:].reshape(n, stride)
    want = oracle_default.decode_batch(cw[:, :223], cw[:, 223:])
    _same((ok.cpu().numpy(), cor.cpu().numpy(), out[:, :223], out[:, 223:255]), want)
    assert (out[:, 255:] == 0).all()  # bytes between rows untouched


@pytest.mark.parametrize("path", ["split", "single"])
@pytest.mark.parametrize("size", [223, 150])
def test_device_separate_parity(monkeypatch, oracle_default, path, size):
    """Data and parity in separate device buffers at odd offsets and strides
    (the syndrome kernel's two-stream path for size 223, its any-alignment
    path for shortened codes): the received parity XORed into the data's
    LFSR parity at every alignment."""
    import torch
    h = _handle(monkeypatch, path)
    rng = np.random.default_rng(size)
    n = 20000
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)
    par = oracle_default.encode_batch(data)
    for c in range(n):
        ne = int(rng.integers(0, 19))
        pos = rng.permutation(size + 32)[:ne]
        mag = rng.integers(1, 256, ne, dtype=np.uint8)
        for p, m in zip(pos, mag):
            if p < size:
                data[c, p] ^= m
            else:
                par[c, p - size] ^= m
    want = oracle_default.decode_batch(data, par)
    ds, ps, do, po = size + 5, 35, 1, 3
    dbuf = np.zeros(do + n * ds, np.uint8)
    pbuf = np.zeros(po + n * ps, np.uint8)
    dbuf[do:].reshape(n, ds)[:, :size] = data
    pbuf[po:].reshape(n, ps)[:, :32] = par
    dd, dp = torch.from_numpy(dbuf).cuda(), torch.from_numpy(pbuf).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    h.decode_batch_device(dd.data_ptr() + do, ds, dp.data_ptr() + po, ps, size, n, ok.data_ptr(), cor.data_ptr(),
                          stream=s)
    torch.cuda.synchronize()
    gd = dd.cpu().numpy()[do:].reshape(n, ds)
    gp = dp.cpu().numpy()[po:].reshape(n, ps)
    _same((ok.cpu().numpy(), cor.cpu().numpy(), gd[:, :size], gp[:, :32]), want)
    assert not gd[:, size:].any() and not gp[:, 32:].any()


def test_split_kernels_timed(monkeypatch, torch_cuda_split):
    """A 2^16 batch with 16 errors each runs the split kernels (timing ids
    1, 4..8) and not the single kernel; the list kernel finds nothing to do."""
    torch = torch_cuda_split
    h = _handle(monkeypatch, "split")
    n = 1 << 16
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    cw = torch.randint(0, 256, (n, 255), dtype=torch.uint8, device="cuda", generator=g)
    s = torch.cuda.current_stream().cuda_stream
    base = cw.data_ptr()
    h.encode_batch_device(base, 255, base + 223, 255, 223, n, s)
    clean = cw.clone()
    pos = torch.rand((n, 255), device="cuda", generator=g).topk(16, dim=1).indices
    mag = torch.randint(1, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    cw.scatter_(1, pos, cw.gather(1, pos) ^ mag)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    h.timing(True)
    h.decode_batch_device(base, 255, base + 223, 255, 223, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    torch.cuda.synchronize()
    t = {k: h.timing_read(k) for k in P.KERNEL_NAMES}
    h.timing(False)
    assert torch.equal(cw, clean) and int(ok.sum()) == n and bool((cor == 16).all())
    for k in (P.KERNEL_REMAINDER, P.KERNEL_BM, P.KERNEL_CHIEN, P.KERNEL_FORNEY, P.KERNEL_APPLY, P.KERNEL_LIST):
        assert t[k][1] == 1, (k, t[k])
    assert t[P.KERNEL_CORRECT][1] == 0


@pytest.fixture(scope="module")
def torch_cuda_split():
    import torch
    assert torch.cuda.is_available()
    return torch


def _erasure_batch(rng, h, n, size, dup):
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    L = size + NR
    slots = np.zeros((n, NR), np.uint8)
    cnt = rng.integers(0, NR + 1, n).astype(np.uint8)
    cnt[: n // 3] = NR  # the configs[3] case, many of them
    for c in range(n):
        e = int(cnt[c])
        slots[c] = rng.permutation(255)[:NR] if c % 5 == 0 else rng.permutation(L)[:NR]  # some past the row
        if c % 2:
            slots[c, :e] = np.sort(slots[c, :e])
        if dup:
            slots[c, e:] = rng.integers(0, 4, NR - e)  # stale slots repeating positions (quirk Q2)
        inrow = slots[c, :e][slots[c, :e] < L]
        cw[c, inrow] ^= rng.integers(1, 256, inrow.size, dtype=np.uint8)
        x = int(rng.integers(0, max(1, (NR - e) // 2 + 2)))
        cw[c, rng.permutation(L)[:x]] ^= rng.integers(1, 256, x, dtype=np.uint8)
    return cw, slots, cnt


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("size,dup", [(223, False), (223, True), (200, False)])
def test_split_erasures_vs_oracle(monkeypatch, oracle_default, path, size, dup):
    """Erasure batches through the record + block-apply path (split) and the
    single kernel: 0..32 slots, sorted and unsorted, slots past the codeword,
    repeated stale slots, extra errors -- bit for bit against the oracle."""
    h = _handle(monkeypatch, path)
    rng = np.random.default_rng(500 + size + dup)
    cw, slots, cnt = _erasure_batch(rng, h, 12000, size, dup)
    got = h.decode_batch(cw[:, :size], cw[:, size:], slots, cnt)
    want = oracle_default.decode_batch(cw[:, :size], cw[:, size:], slots.astype(np.uint32), cnt.astype(np.uint32))
    assert want[0].sum() > 1000
    _same(got, want)


def test_split_erasure_kernels_timed(monkeypatch, torch_cuda_split):
    """A 2^16 batch with 32 sorted erasures each: remainder, rs_era_bp_k, the
    (empty) list, block apply -- codewords restored, 32 corrections each."""
    torch = torch_cuda_split
    h = _handle(monkeypatch, "split")
    n = 1 << 16
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    cw = torch.randint(0, 256, (n, 255), dtype=torch.uint8, device="cuda", generator=g)
    s = torch.cuda.current_stream().cuda_stream
    base = cw.data_ptr()
    h.encode_batch_device(base, 255, base + 223, 255, 223, n, s)
    clean = cw.clone()
    pos = torch.rand((n, 223), device="cuda", generator=g).topk(NR, dim=1).indices.sort(dim=1).values
    mag = torch.randint(1, 256, (n, NR), dtype=torch.uint8, device="cuda", generator=g)
    cw.scatter_(1, pos, cw.gather(1, pos) ^ mag)
    slots = pos.to(torch.uint8).contiguous()
    cnt = torch.full((n,), NR, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    h.timing(True)
    h.decode_batch_device(base, 255, base + 223, 255, 223, n, ok.data_ptr(), cor.data_ptr(),
                          d_positions=slots.data_ptr(), positions_stride=NR, d_counts=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    t = {k: h.timing_read(k) for k in P.KERNEL_NAMES}
    h.timing(False)
    assert torch.equal(cw, clean) and int(ok.sum()) == n and bool((cor == NR).all())
    for k in (P.KERNEL_REMAINDER, P.KERNEL_ERASURE, P.KERNEL_LIST, P.KERNEL_APPLY):
        assert t[k][1] == 1, (k, t[k])
    assert t[P.KERNEL_CORRECT][1] == 0


@pytest.mark.parametrize("params", [(8, 0x11D, 0, 1, 32), (8, 0x187, 5, 1, 32), (8, 0x11D, 1, 2, 32),
                                    (8, 0x11D, 5, 7, 32)])
def test_split_erasures_other_parameters_vs_oracle(monkeypatch, params):
    """Erasure batches under other fcr / prim / field polynomials: rs_era_bp_k
    (prim 1, any fcr) and the record-mode general kernel (prim != 1)."""
    from oracle import Oracle
    o = Oracle(*params)
    h = _handle(monkeypatch, "split", params)
    rng = np.random.default_rng(sum(params) + 7)
    cw, slots, cnt = _erasure_batch(rng, h, 9000, 223, False)
    got = h.decode_batch(cw[:, :223], cw[:, 223:], slots, cnt)
    want = o.decode_batch(cw[:, :223], cw[:, 223:], slots.astype(np.uint32), cnt.astype(np.uint32))
    assert want[0].sum() > 1000
    _same(got, want)


@pytest.mark.parametrize("path", PATHS)
def test_erasure_count_past_roots(monkeypatch, oracle_default, path):
    """Erasure counts 33..255 (quirk Q5, undefined in the reference only once
    the locator is built): a clean codeword succeeds with 0 corrections
    whatever its count (src/decode.c:468 tests the syndromes first), a dirty
    one is refused (ok 0, bytes untouched) -- the same answer on the split
    path (rs_era_bp_k + list) and the single kernel, mixed with in-range
    codewords in every wave."""
    h = _handle(monkeypatch, path)
    rng = np.random.default_rng(4242)
    n = 16384
    data = rng.integers(0, 256, (n, 223), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    slots = np.zeros((n, NR), np.uint8)
    cnt = rng.integers(33, 256, n).astype(np.uint8)
    inr = np.arange(n) % 3 == 0  # in-range codewords: 32 sorted erasures
    cnt[inr] = NR
    dirty = np.arange(n) % 2 == 0
    for c in range(n):
        slots[c] = np.sort(rng.permutation(223)[:NR])
        if dirty[c]:
            cw[c, slots[c]] ^= rng.integers(1, 256, NR, dtype=np.uint8)
    ok, cor, d, p = h.decode_batch(cw[:, :223], cw[:, 223:], slots, cnt)
    clean_far = ~dirty & ~inr
    dirty_far = dirty & ~inr
    assert (ok[clean_far] == 1).all() and (cor[clean_far] == 0).all()
    assert (ok[dirty_far] == 0).all() and (cor[dirty_far] == 0).all()
    out = np.concatenate([d, p], 1)
    assert (out[~inr] == cw[~inr]).all()
    want = oracle_default.decode_batch(cw[inr, :223], cw[inr, 223:], slots[inr].astype(np.uint32),
                                       cnt[inr].astype(np.uint32))
    _same((ok[inr], cor[inr], d[inr], p[inr]), want)


def _errata_batch(rng, h, n, size, ne, nerr, sort=True, mag=None):
    """ne erasures (slots in the message, sorted or in insertion order, stale
    slots after the count) and 0..nerr errors elsewhere in each codeword."""
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    L = size + NR
    slots = np.zeros((n, NR), np.uint8)
    cnt = np.full(n, ne, np.uint8)
    for c in range(n):
        er = rng.permutation(size)[:ne]
        if sort:
            er = np.sort(er)
        slots[c, :ne] = er
        slots[c, ne:] = rng.integers(0, L, NR - ne)  # stale entries past the count (quirk Q1)
        cw[c, er] ^= rng.integers(1, 256, ne, dtype=np.uint8) if mag is None else np.uint8(mag)
        x = int(rng.integers(0, nerr + 1))
        rest = np.setdiff1d(np.arange(L), er)
        cw[c, rng.permutation(rest)[:x]] ^= rng.integers(1, 256, x, dtype=np.uint8)
    return cw, slots, cnt


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("size,ne,nerr,sort,mag", [
    (223, 16, 8, True, None),   # errors and erasures: the errata kernels' target case
    (223, 16, 0, False, 0xFF),  # tests/test_codec.c:123-168: 16 erasures in insertion order, magnitude 0xFF
    (64, 20, 0, False, 0xFF),   # tests/test_unified.c:82-112: 20 erasures in a 64-byte message
    (223, 24, 4, True, None),
    (223, 8, 12, False, None),
    (200, 16, 8, True, None),
    (223, 31, 0, True, None),
    (223, 1, 15, True, None)])
def test_errata_vs_oracle(monkeypatch, oracle_default, path, size, ne, nerr, sort, mag):
    """Erasure counts below 32 with errors besides (rs_ebm_k, rs_chien32_k,
    rs_forney32_k, then the record apply) and the single kernel, bit for bit
    against the oracle -- including the reference's own erasure test cases,
    whose codewords come back restored."""
    h = _handle(monkeypatch, path)
    rng = np.random.default_rng(700 + size + ne * 3 + nerr)
    cw, slots, cnt = _errata_batch(rng, h, 10000, size, ne, nerr, sort, mag)
    got = h.decode_batch(cw[:, :size], cw[:, size:], slots, cnt)
    want = oracle_default.decode_batch(cw[:, :size], cw[:, size:], slots.astype(np.uint32), cnt.astype(np.uint32))
    assert want[0].sum() > 9000
    _same(got, want)
    if mag is not None:  # the reference tests' assertion: the message is restored
        assert got[0].all()


def test_errata_kernels_timed(monkeypatch, torch_cuda_split):
    """2^16 codewords with 16 sorted erasures and 8 errors each on the device
    API: rs_era_bp_k leaves them pending, the errata kernels decode them, the
    general kernel never runs; ok / corrected for all, bytes of a sample
    against the oracle."""
    torch = torch_cuda_split
    from oracle import Oracle
    o = Oracle(8, 0x11D, 1, 1, 32)
    h = _handle(monkeypatch, "split")
    n = 1 << 16
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    cw = torch.randint(0, 256, (n, 255), dtype=torch.uint8, device="cuda", generator=g)
    s = torch.cuda.current_stream().cuda_stream
    base = cw.data_ptr()
    h.encode_batch_device(base, 255, base + 223, 255, 223, n, s)
    r = torch.rand((n, 255), device="cuda", generator=g)
    era = r[:, :223].topk(16, dim=1).indices.sort(dim=1).values  # erasures in the message
    pos = r.scatter(1, era, -1.0).topk(8, dim=1).indices  # errors anywhere else
    mag = torch.randint(1, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    cw.scatter_(1, era, cw.gather(1, era) ^ mag)
    emag = torch.randint(1, 256, (n, 8), dtype=torch.uint8, device="cuda", generator=g)
    cw.scatter_(1, pos, cw.gather(1, pos) ^ emag)
    slots = torch.zeros((n, NR), dtype=torch.uint8, device="cuda")
    slots[:, :16] = era.to(torch.uint8)
    cnt = torch.full((n,), 16, dtype=torch.uint8, device="cuda")
    before = cw.cpu().numpy()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    h.timing(True)
    h.decode_batch_device(base, 255, base + 223, 255, 223, n, ok.data_ptr(), cor.data_ptr(),
                          d_positions=slots.data_ptr(), positions_stride=NR, d_counts=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    t = {k: h.timing_read(k) for k in P.KERNEL_NAMES}
    h.timing(False)
    for k in (P.KERNEL_REMAINDER, P.KERNEL_ERASURE, P.KERNEL_BM, P.KERNEL_CHIEN, P.KERNEL_FORNEY, P.KERNEL_LIST,
              P.KERNEL_APPLY):
        assert t[k][1] == 1, (k, t[k])
    assert t[P.KERNEL_CORRECT][1] == 0
    assert int(ok.sum()) == n
    sel = np.arange(0, n, 29)
    sl = slots.cpu().numpy()[sel].astype(np.uint32)
    want = o.decode_batch(before[sel, :223], before[sel, 223:], sl, np.full(sel.size, 16, np.uint32))
    out = cw.cpu().numpy()[sel]
    _same((ok.cpu().numpy()[sel], cor.cpu().numpy()[sel], out[:, :223], out[:, 223:]), want)


@pytest.mark.parametrize("stride", [32, 40, 33])
def test_errata_slot_strides(monkeypatch, oracle_default, torch_cuda_split, stride):
    """Slot rows 32 (rs_era_bp_k + errata), 40 (errata alone: not 16-byte rows)
    and 33 bytes apart (unaligned rows: the general kernel) give the same
    answers, equal to the oracle's."""
    torch = torch_cuda_split
    h = _handle(monkeypatch, "split")
    rng = np.random.default_rng(stride)
    cw, slots, cnt = _errata_batch(rng, h, 9000, 223, 12, 10, sort=bool(stride & 1))
    want = oracle_default.decode_batch(cw[:, :223], cw[:, 223:], slots.astype(np.uint32), cnt.astype(np.uint32))
    n = cw.shape[0]
    d = torch.from_numpy(cw.copy()).cuda()
    sl = np.zeros((n, stride), np.uint8)
    sl[:, :NR] = slots
    sd = torch.from_numpy(sl.reshape(-1)).cuda()
    cd = torch.from_numpy(cnt).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    base = d.data_ptr()
    h.decode_batch_device(base, 255, base + 223, 255, 223, n, ok.data_ptr(), cor.data_ptr(),
                          d_positions=sd.data_ptr(), positions_stride=stride, d_counts=cd.data_ptr(), stream=s)
    torch.cuda.synchronize()
    out = d.cpu().numpy()
    _same((ok.cpu().numpy(), cor.cpu().numpy(), out[:, :223], out[:, 223:]), want)
