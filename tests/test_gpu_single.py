"""GPU parity of the one-codeword decoder (rs_single.hip: rs_dec1_k, rs_enc1_k),
which serves every poporon_decode / poporon_encode call of a default-field
handle and every device batch of one codeword.

Expected values: the CPU oracle (oracle/rs_oracle.c, pinned to the golden
fixtures of the compiled reference) on the same seeded inputs, compared
bit-exactly: bytes, the bool result and corrected_num -- over random error
counts up to and past capacity (failures and the reference's
miscorrections), erasure lists (sorted, unsorted, stale slots past the count,
slots past the codeword, extra errors), external syndromes, shortened codes
and other fcr / prim / field polynomials.
"""
import numpy as np
import pytest

import libpoporon_amd as P

pytestmark = pytest.mark.gpu

NR = 32
PARAMS = [(8, 0x11D, 1, 1, 32), (8, 0x11D, 0, 1, 32), (8, 0x187, 5, 1, 32), (8, 0x11D, 1, 2, 32),
          (8, 0x11D, 5, 7, 32)]


def _need_gpu():
    if P.device_count() == 0:
        pytest.fail("no HIP device: GPU tests must run on the MI355X box")


@pytest.mark.parametrize("params", PARAMS)
@pytest.mark.parametrize("size", [223, 120, 1])
def test_single_decode_random_vs_oracle(params, size):
    """0..28 random errors per codeword (clean, correctable, beyond capacity)."""
    _need_gpu()
    from oracle import Oracle
    o = Oracle(*params)
    h = P.Poporon(*params)
    rng = np.random.default_rng(sum(params) * 1000 + size)
    L = size + NR
    n = 400
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)
    par = o.encode_batch(data)
    for c in range(n):
        assert (h.encode(data[c]) == par[c]).all(), c
        cw = np.concatenate([data[c], par[c]])
        ne = int(rng.integers(0, min(29, L + 1)))
        pos = rng.permutation(L)[:ne]
        cw[pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
        got = h.decode(cw[:size], cw[size:])
        want = o.decode(cw[:size], cw[size:])
        assert got[0] == want[0] and got[1] == want[1], (c, ne, got[:2], want[:2])
        assert (got[2] == want[2]).all() and (got[3] == want[3]).all(), c


@pytest.mark.parametrize("params", PARAMS[:3])
def test_single_erasures_vs_oracle(params):
    """Erasure object attached: 0..32 slots (sorted or not, some past the
    codeword), stale slots past the count (quirks Q1/Q2), extra errors."""
    _need_gpu()
    from oracle import Oracle
    o = Oracle(*params)
    er = P.Erasure(32, 32)
    h = P.Poporon(*params, erasure=er)
    rng = np.random.default_rng(sum(params) + 99)
    n = 500
    size = 223
    L = size + NR
    data = rng.integers(0, 256, (n, size), dtype=np.uint8)
    par = o.encode_batch(data)
    nok = 0
    for c in range(n):
        cw = np.concatenate([data[c], par[c]])
        e = int(rng.integers(0, NR + 1))
        slots = (rng.permutation(L) if c % 7 else rng.permutation(255))[:NR].astype(np.uint32)
        if c % 2:
            slots[:e] = np.sort(slots[:e])
        inrow = slots[:e][slots[:e] < L]
        cw[inrow] ^= rng.integers(1, 256, inrow.size, dtype=np.uint8)
        x = int(rng.integers(0, max(1, (NR - e) // 2 + 2)))
        cw[rng.permutation(L)[:x]] ^= rng.integers(1, 256, x, dtype=np.uint8)
        er.set(slots)         # stale slots beyond the count
        er.set(slots[:e])
        got = h.decode(cw[:size], cw[size:])
        wok, wcor, wd, wp = o.decode_batch(cw[None, :size], cw[None, size:], slots[None], np.array([e], np.uint32))
        assert got[0] == bool(wok[0]) and got[1] == int(wcor[0]), (c, e, x, got[:2], wok, wcor)
        assert (got[2] == wd[0]).all() and (got[3] == wp[0]).all(), c
        nok += got[0]
    assert nok > n // 4


def test_single_erasure_count_past_roots():
    """More erasures than roots (quirk Q5): clean codeword -> success, dirty
    -> refused with the bytes untouched, as the batch kernels."""
    _need_gpu()
    er = P.Erasure(32, 32)
    h = P.Poporon(8, 0x11D, 1, 1, 32, erasure=er)
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 223, dtype=np.uint8)
    par = h.encode(data)
    er.set(range(40))
    ok, n, d, p = h.decode(data, par)
    assert ok and n == 0 and (d == data).all() and (p == par).all()
    bad = data.copy()
    bad[3] ^= 0x55
    ok, n, d, p = h.decode(bad, par)
    assert not ok and n == 0 and (d == bad).all() and (p == par).all()


def test_single_external_syndromes_vs_oracle():
    """External log-form syndromes (src/decode.c:446-464): the syndromes of
    corrupted codewords, all-zero (255) syndromes, random syndromes, and
    out-of-table values (> 255: refused)."""
    _need_gpu()
    from oracle import Oracle
    o = Oracle()
    rng = np.random.default_rng(31)
    for c in range(120):
        data = rng.integers(0, 256, 223, dtype=np.uint8)
        cw = np.concatenate([data, o.encode(data)])
        ne = int(rng.integers(0, 20))
        cw[rng.permutation(255)[:ne]] ^= rng.integers(1, 256, ne, dtype=np.uint8)
        if c % 4 == 0:
            syn = np.full(NR, 255, np.uint16)
        elif c % 4 == 1:
            syn = rng.integers(0, 256, NR).astype(np.uint16)
        else:
            syn = o.syndrome(cw[:223], cw[223:])[1]
        h = P.Poporon(8, 0x11D, 1, 1, 32, syndrome=syn)
        got = h.decode(cw[:223], cw[223:])
        want = o.decode(cw[:223], cw[223:], ext_syn=syn)
        assert got[0] == want[0] and got[1] == want[1], (c, got[:2], want[:2])
        assert (got[2] == want[2]).all() and (got[3] == want[3]).all(), c
        h.close()
    syn = np.full(NR, 255, np.uint16)
    syn[7] = 300
    h = P.Poporon(8, 0x11D, 1, 1, 32, syndrome=syn)
    ok, n, d, _ = h.decode(cw[:223], cw[223:])
    assert not ok and n == 0 and (d == cw[:223]).all()


def test_batch_of_one_device(oracle_default):
    """A device batch of one codeword runs rs_dec1_k with device pointers (u8
    slots and counts in erasure mode)."""
    _need_gpu()
    h = P.Poporon.default()
    rng = np.random.default_rng(12)
    for c in range(60):
        data = rng.integers(0, 256, (1, 223), dtype=np.uint8)
        cw = np.concatenate([data, oracle_default.encode_batch(data)], 1)
        if c % 2:
            ne = int(rng.integers(0, 22))
            cw[0, rng.permutation(255)[:ne]] ^= rng.integers(1, 256, ne, dtype=np.uint8)
            got = h.decode_batch(cw[:, :223], cw[:, 223:])
            want = oracle_default.decode_batch(cw[:, :223], cw[:, 223:])
        else:
            e = int(rng.integers(0, 33))
            slots = np.sort(rng.permutation(223)[:NR]).astype(np.uint8)[None]
            cw[0, slots[0, :e]] ^= rng.integers(1, 256, e, dtype=np.uint8)
            cnt = np.array([e], np.uint8)
            got = h.decode_batch(cw[:, :223], cw[:, 223:], slots, cnt)
            want = oracle_default.decode_batch(cw[:, :223], cw[:, 223:], slots.astype(np.uint32),
                                               cnt.astype(np.uint32))
        for g, w in zip(got, want):
            assert (np.asarray(g) == np.asarray(w)).all(), c
    h.timing(True)
    h.decode_batch(cw[:, :223], cw[:, 223:])
    t = {k: h.timing_read(k) for k in P.KERNEL_NAMES}
    h.timing(False)
    assert t[P.KERNEL_SINGLE][1] == 1 and t[P.KERNEL_CORRECT][1] == 0 and t[P.KERNEL_REMAINDER][1] == 0


@pytest.mark.parametrize("n", [1, 2, 300, 16384])
def test_batch_device_without_corrected(oracle_default, n):
    """poporon_decode_batch_device with d_corrected NULL (optional in the
    header) on each batch route: rs_dec1_k (1), rs_wave_k (2, 300) and the
    split kernels (16384)."""
    _need_gpu()
    import torch
    h = P.Poporon.default()
    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, (n, 223), dtype=np.uint8)
    cw = np.concatenate([data, oracle_default.encode_batch(data)], 1)
    for i in range(n):
        cw[i, rng.permutation(255)[:16]] ^= rng.integers(1, 256, 16, dtype=np.uint8)
    want = oracle_default.decode_batch(cw[:, :223], cw[:, 223:])
    d = torch.from_numpy(cw).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    b = d.data_ptr()
    h.decode_batch_device(b, 255, b + 223, 255, 223, n, ok.data_ptr(), None)
    torch.cuda.synchronize()
    assert (ok.cpu().numpy() == np.asarray(want[0]).astype(np.uint8)).all()
    assert (d.cpu().numpy()[:, :223] == np.asarray(want[2])).all()


def test_single_call_many(oracle_default):
    """2000 back-to-back poporon_encode / poporon_decode calls (the latency
    path: completion words polled in host memory), 16 errors each."""
    _need_gpu()
    h = P.Poporon.default()
    rng = np.random.default_rng(77)
    msgs = rng.integers(0, 256, (2000, 223), dtype=np.uint8)
    want_par = oracle_default.encode_batch(msgs)
    for c in range(2000):
        p = h.encode(msgs[c])
        assert (p == want_par[c]).all(), c
        cw = np.concatenate([msgs[c], p])
        cw[rng.permutation(255)[:16]] ^= rng.integers(1, 256, 16, dtype=np.uint8)
        ok, n, d, q = h.decode(cw[:223], cw[223:])
        assert ok and n == 16 and (d == msgs[c]).all() and (q == p).all(), c


def test_single_call_server_idle_and_relaunch(oracle_default):
    """The single-call server (rs_serve_k) leaves after 1 ms without a
    request and is launched again by the next call; calls spaced around that
    limit, device batches and device synchronisations in between, and a
    second handle serving at the same time all give the oracle's bytes."""
    import time

    import torch
    _need_gpu()
    h, h2 = P.Poporon.default(), P.Poporon.default()
    rng = np.random.default_rng(2024)
    msgs = rng.integers(0, 256, (48, 223), dtype=np.uint8)
    want = oracle_default.encode_batch(msgs)
    for c in range(48):
        if c % 3 == 0:
            time.sleep([0.0, 0.0009, 0.0011, 0.003][(c // 3) % 4])  # around the 1 ms idle limit
        if c % 8 == 5:
            torch.cuda.synchronize()  # waits for a live server to leave (at most its idle limit)
        if c % 8 == 6:
            got = h.decode_batch(np.tile(msgs[c], (3, 1)), np.tile(want[c], (3, 1)))  # a device batch between calls
            assert got[0].all()
        hh = h if c % 2 else h2
        assert (hh.encode(msgs[c]) == want[c]).all(), c
        cw = np.concatenate([msgs[c], want[c]])
        cw[rng.permutation(255)[:16]] ^= rng.integers(1, 256, 16, dtype=np.uint8)
        ok, n, d, q = hh.decode(cw[:223], cw[223:])
        assert ok and n == 16 and (d == msgs[c]).all() and (q == want[c]).all(), c
    h.close()  # asks a live server to leave at once
    assert (h2.encode(msgs[0]) == want[0]).all()


def test_batch_after_single_call(oracle_default):
    """A device batch issued right after a single call: the batch entry point
    first asks the handle's live server to leave (api.cpp srv_stop), so the
    batch is not left waiting for the CU the server holds.  Results equal the
    ones without a single call before them, and the batch takes no longer
    than 1.5x + 0.2 ms of that (tools/server_batch.py measures the same)."""
    import time

    import torch
    _need_gpu()
    h = P.Poporon.default()
    n = 1 << 20
    rng = np.random.default_rng(9)
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 223), dtype=np.uint8)).cuda()
    par = torch.zeros((n, NR), dtype=torch.uint8, device="cuda")
    one = msgs[0].cpu().numpy()
    want_one = oracle_default.encode_batch(one[None])[0]
    s = torch.cuda.current_stream().cuda_stream
    times = {True: [], False: []}
    ref = None
    for r in range(12):
        after = bool(r % 2)
        if after:
            assert (h.encode(one) == want_one).all()  # the server is resident now
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.encode_batch_device(msgs.data_ptr(), 223, par.data_ptr(), NR, 223, n, s)
        torch.cuda.synchronize()
        times[after].append(time.perf_counter() - t0)
        if ref is None:
            ref = par.clone()
        assert torch.equal(par, ref), r
    sample = msgs[::4096].cpu().numpy()
    assert (oracle_default.encode_batch(sample) == ref[::4096].cpu().numpy()).all()
    alone, after = np.median(times[False][1:]), np.median(times[True][1:])
    assert after <= 1.5 * alone + 2e-4, (alone, after)
