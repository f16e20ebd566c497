"""GPU tests: full-size configurations, the syndrome API, multi-GPU C ABI,
workspace ordering across streams, the test utilities and the compiled C
drop-in programs.  Everything goes through libpoporon_amd.so (C ABI).

Full sizes use size-independent properties (every codeword decodes back to
the encoded word with ok = 1 and corrected = 16 / 32; an order-independent
checksum of the decoded batch equals that of the encoded batch) plus a
1-in-4096 sample compared bit for bit with the CPU oracle.
"""
import os
import subprocess

import numpy as np
import pytest

import libpoporon_amd as P
import testutil as T

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, NR, N = 223, 32, 255
SEED = 0x5EED0001


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.fixture(scope="module")
def rs():
    if P.device_count() == 0:
        pytest.fail("no HIP device: GPU tests must run on the MI355X box")
    return P.Poporon.default()


def _stream(torch):
    return torch.cuda.current_stream().cuda_stream


def _checksum(torch, rows, first=0):
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    T.checksum(rows.data_ptr(), N, N, first, rows.shape[0], s.data_ptr(), _stream(torch))
    return int(s.item()) & ((1 << 64) - 1)


def _synth(torch, n, seed=SEED, first=0):
    rows = torch.empty((n, N), dtype=torch.uint8, device="cuda")
    T.synth_rows(seed, first, n, K, rows.data_ptr(), N, _stream(torch))
    return rows


def _errors(torch, n, nerr, span, seed, sorted_positions=False, first=0):
    pos = torch.empty((n, nerr), dtype=torch.uint8, device="cuda")
    mag = torch.empty((n, nerr), dtype=torch.uint8, device="cuda")
    T.synth_errors(seed, first, n, nerr, span, pos.data_ptr(), mag.data_ptr(), sorted_positions, _stream(torch))
    return pos, mag


# ---------------------------------------------------------------------------
# test utilities: the HIP kernels equal their numpy restatements
# ---------------------------------------------------------------------------
def test_testutil_matches_numpy(torch_cuda):
    torch = torch_cuda
    n, first = 3000, 123457
    rows = _synth(torch, n, first=first)
    torch.cuda.synchronize()
    host = rows.cpu().numpy()
    assert (host[:, :K] == T.synth_rows_cpu(SEED, first, n, K)).all()
    for nerr, span, srt in ((16, 255, False), (32, 223, True), (5, 17, False)):
        pos, mag = _errors(torch, n, nerr, span, SEED + 9, srt, first=first)
        torch.cuda.synchronize()
        wp, wm = T.synth_errors_cpu(SEED + 9, first, n, nerr, span, srt)
        assert (pos.cpu().numpy() == wp).all() and (mag.cpu().numpy() == wm).all(), (nerr, span, srt)
    host[:, K:] = np.random.default_rng(1).integers(0, 256, (n, NR), dtype=np.uint8)
    rows.copy_(torch.from_numpy(host).cuda())
    pos, mag = _errors(torch, n, 16, 255, SEED + 1, first=first)
    T.channel_xor(pos.data_ptr(), mag.data_ptr(), 16, rows.data_ptr(), N, n, _stream(torch))
    torch.cuda.synchronize()
    want = T.channel_xor_cpu(host, pos.cpu().numpy(), mag.cpu().numpy())
    assert (rows.cpu().numpy() == want).all()
    assert _checksum(torch, rows, first) == T.checksum_cpu(want, first)


# ---------------------------------------------------------------------------
# syndromes (calculate_syndrome_u8 per codeword) against the reference
# ---------------------------------------------------------------------------
def _syndromes(torch, h, rows_np, size, nr):
    n = rows_np.shape[0]
    t = torch.from_numpy(np.ascontiguousarray(rows_np)).cuda()
    syn = torch.zeros((n, nr), dtype=torch.int16, device="cuda")  # uint16 bit patterns
    nz = torch.zeros(n, dtype=torch.uint8, device="cuda")
    w = size + nr
    h.syndrome_batch_device(t.data_ptr(), w, t.data_ptr() + size, w, size, n, syn.data_ptr(), nr, nz.data_ptr(),
                            _stream(torch))
    torch.cuda.synchronize()
    return syn.cpu().numpy().astype(np.uint16), nz.cpu().numpy()


def test_syndromes_golden(rs, golden, torch_cuda):
    """The kernel's syndromes equal the ones the compiled reference computed
    for every golden decode case (dec_syn: u16 log form, 255 = zero)."""
    sizes = golden["dec_size"]
    for s in np.unique(sizes):
        sel = np.nonzero(sizes == s)[0]
        s = int(s)
        syn, nz = _syndromes(torch_cuda, rs, golden["dec_in"][sel, :s + NR], s, NR)
        want = golden["dec_syn"][sel]
        assert (syn == want).all(), s
        assert (nz == (want != 255).any(axis=1)).all(), s


@pytest.mark.parametrize("params", [(8, 0x11D, 1, 1, 32), (8, 0x187, 112, 11, 32), (8, 0x11D, 1, 1, 16),
                                    (6, 0x43, 1, 1, 10), (4, 0x13, 1, 2, 8)])
def test_syndromes_vs_oracle(torch_cuda, params):
    from oracle import Oracle
    m, poly, fcr, prim, nr = params
    o, h = Oracle(*params), P.Poporon(*params)
    nn = (1 << m) - 1
    rng = np.random.default_rng(sum(params))
    for size in (nn - nr, max(1, (nn - nr) // 3)):
        data = rng.integers(0, nn + 1, (500, size), dtype=np.uint8)
        cw = np.concatenate([data, o.encode_batch(data)], 1)
        for c in range(1, 500):
            ne = c % (nr + 3)
            p = rng.permutation(size + nr)[:ne]
            cw[c, p] ^= rng.integers(1, nn + 1, ne).astype(np.uint8)
        syn, nz = _syndromes(torch_cuda, h, cw, size, nr)
        for c in range(500):
            f, s = o.syndrome(cw[c, :size], cw[c, size:])
            assert (syn[c] == s).all() and bool(nz[c]) == f, (size, c)


# ---------------------------------------------------------------------------
# one handle, two streams: the syndrome workspace is ordered across streams
# ---------------------------------------------------------------------------
def test_one_handle_two_streams(torch_cuda):
    """Back-to-back decode_batch_device calls of ONE handle on two streams
    share the handle's workspace; the second call's stream waits for the
    first call's last reader (poporon_amd.h), so both batches decode right."""
    torch = torch_cuda
    h = P.Poporon.default()
    n = 1 << 18
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    bufs, cleans, sts = [], [], []
    for k in range(2):
        rows = _synth(torch, n, seed=SEED + 20 + k)
        b = rows.data_ptr()
        h.encode_batch_device(b, N, b + K, N, K, n, _stream(torch))
        cleans.append(rows.clone())
        pos, mag = _errors(torch, n, 16, N, SEED + 30 + k)
        T.channel_xor(pos.data_ptr(), mag.data_ptr(), 16, b, N, n, _stream(torch))
        bufs.append(rows)
        sts.append((torch.zeros(n, dtype=torch.uint8, device="cuda"), torch.zeros(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    for k, s in enumerate((s1, s2)):  # enqueued back to back, no host sync in between
        b = bufs[k].data_ptr()
        h.decode_batch_device(b, N, b + K, N, K, n, sts[k][0].data_ptr(), sts[k][1].data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    for k in range(2):
        assert bool((sts[k][0] == 1).all()) and bool((sts[k][1] == 16).all())
        assert torch.equal(bufs[k], cleans[k])


# ---------------------------------------------------------------------------
# full sizes: configs[4]'s per-GPU share at 8 GPUs (2^23), all of configs[4]
# on one GPU (2^26 codewords, 16.3 GB), configs[3] at 2^20
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1 << 23, 1 << 26])
def test_full_size_roundtrip(rs, oracle_default, torch_cuda, n):
    torch = torch_cuda
    rows = _synth(torch, n, seed=SEED + 4)
    b = rows.data_ptr()
    s = _stream(torch)
    rs.encode_batch_device(b, N, b + K, N, K, n, s)
    torch.cuda.synchronize()
    sample = rows[::4096].cpu().numpy()
    assert (oracle_default.encode_batch(sample[:, :K]) == sample[:, K:]).all()
    clean_sum = _checksum(torch, rows)
    pos, mag = _errors(torch, n, 16, N, SEED + 5)
    T.channel_xor(pos.data_ptr(), mag.data_ptr(), 16, b, N, n, s)
    del pos, mag
    torch.cuda.synchronize()
    bad_sample = rows[::4096].cpu().numpy()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert int((ok != 1).sum()) == 0
    assert int((cor != 16).sum()) == 0
    assert _checksum(torch, rows) == clean_sum
    ook, ocor, od, op = oracle_default.decode_batch(bad_sample[:, :K], bad_sample[:, K:])
    got = rows[::4096].cpu().numpy()
    assert (ook == 1).all() and (ocor == 16).all()
    assert (got[:, :K] == od).all() and (got[:, K:] == op).all()


def test_erasure_full_size(rs, oracle_default, torch_cuda):
    """configs[3]: 2^20 codewords, 32 sorted erasures in [0, 223) each."""
    torch = torch_cuda
    n = 1 << 20
    rows = _synth(torch, n, seed=SEED + 6)
    b = rows.data_ptr()
    s = _stream(torch)
    rs.encode_batch_device(b, N, b + K, N, K, n, s)
    torch.cuda.synchronize()
    clean_sum = _checksum(torch, rows)
    slots, mag = _errors(torch, n, 32, K, SEED + 2, sorted_positions=True)
    T.channel_xor(slots.data_ptr(), mag.data_ptr(), 32, b, N, n, s)
    torch.cuda.synchronize()
    bad_sample = rows[::4096].cpu().numpy()
    slot_sample = slots[::4096].cpu().numpy()
    cnt = torch.full((n,), 32, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")
    rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), d_positions=slots.data_ptr(),
                           positions_stride=32, d_counts=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert int((ok != 1).sum()) == 0 and int((cor != 32).sum()) == 0
    assert _checksum(torch, rows) == clean_sum
    m = bad_sample.shape[0]
    ook, ocor, od, op = oracle_default.decode_batch(bad_sample[:, :K], bad_sample[:, K:], slot_sample.astype(np.uint32),
                                                    np.full(m, 32, np.uint32))
    got = rows[::4096].cpu().numpy()
    assert (got[:, :K] == od).all() and (got[:, K:] == op).all() and (ocor == 32).all()


# ---------------------------------------------------------------------------
# multi-GPU C ABI (every visible device; one on the test box)
# ---------------------------------------------------------------------------
def test_multi_device_api(oracle_default, torch_cuda):
    torch = torch_cuda
    m = P.Multi()
    G = m.devices
    assert G == P.device_count() >= 1
    rng = np.random.default_rng(404)
    n = 20000
    data = rng.integers(0, 256, (n, K), dtype=np.uint8)
    par = m.encode_batch(data)
    assert (par == oracle_default.encode_batch(data)).all()
    cw = np.concatenate([data, par], 1)
    for c in range(n):
        ne = c % 20
        p = rng.permutation(N)[:ne]
        cw[c, p] ^= rng.integers(1, 256, ne, dtype=np.uint8)
    ok, cor, d, p = m.decode_batch(cw[:, :K], cw[:, K:])
    ook, ocor, od, op = oracle_default.decode_batch(cw[:, :K], cw[:, K:])
    assert (ok == ook).all() and (cor == ocor).all() and (d == od).all() and (p == op).all()
    # device-resident shards: device i holds rows [first_i, first_i + n_i)
    shards, oks, cors, ptrs = [], [], [], []
    for i in range(G):
        lo, hi = P.shard_range(n, i, G)
        with torch.cuda.device(i):
            t = torch.from_numpy(np.ascontiguousarray(cw[lo:hi])).to(f"cuda:{i}")
            shards.append(t)
            oks.append(torch.zeros(hi - lo, dtype=torch.uint8, device=f"cuda:{i}"))
            cors.append(torch.zeros(hi - lo, dtype=torch.uint8, device=f"cuda:{i}"))
    for i in range(G):
        torch.cuda.synchronize(i)
    m.decode_batch_device([t.data_ptr() for t in shards], N, [t.data_ptr() + K for t in shards], N, K, n,
                          [o.data_ptr() for o in oks], [c.data_ptr() for c in cors])
    for i in range(G):
        torch.cuda.synchronize(i)
    out = np.concatenate([t.cpu().numpy() for t in shards])
    assert (np.concatenate([o.cpu().numpy() for o in oks]) == ook).all()
    assert (np.concatenate([c.cpu().numpy() for c in cors]) == ocor).all()
    assert (out[:, :K] == od).all() and (out[:, K:] == op).all()
    m.close()


def _mixed_channel(rng, n):
    """Codewords with errors only (even c: 0..19 errors, past t as well) and
    erasure rows (odd c: 0, 8, 16 or 32 sorted slots in the data, plus errors
    within 2e + era <= 32); slots past the count stay 0 (read by the
    reference as stale entries, quirk Q2)."""
    data = rng.integers(0, 256, (n, K), dtype=np.uint8)
    slots = np.zeros((n, NR), np.uint8)
    cnts = np.zeros(n, np.uint8)
    errs = []
    for c in range(n):
        era = (0, 8, 16, 32)[(c >> 1) % 4] if c % 2 else 0
        if era:
            slots[c, :era] = np.sort(rng.choice(K, era, replace=False))
            cnts[c] = era
        ne = (NR - era) // 2 if c % 2 else c % 20
        errs.append((era, ne))
    return data, slots, cnts, errs


@pytest.mark.parametrize("G", [2, 4, 8])
def test_multi_device_repeated(oracle_default, torch_cuda, G):
    """The multi-device C ABI at G > 1 on one GPU: G independent handles on
    device 0, each taking its contiguous range (poporon_amd_multi_range), the
    host entry points with one host thread per handle and the device entry
    points with per-handle shards and streams.  Bytes, ok and corrected_num
    equal the oracle's for error and erasure batches.  At G = 2 each handle's
    range (20,000 codewords) takes the split kernels, at G = 4 / 8 (10,000 /
    5,000) the one-codeword-per-wave kernel."""
    torch = torch_cuda
    m = P.Multi(devices=[0] * G)
    assert m.devices == G
    n = 80000
    rng = np.random.default_rng(500 + G)
    data, slots, cnts, errs = _mixed_channel(rng, n)
    par = m.encode_batch(data)
    assert (par == oracle_default.encode_batch(data)).all()
    cw = np.concatenate([data, par], 1)
    for c, (era, ne) in enumerate(errs):
        for s in slots[c, :era]:
            cw[c, s] ^= rng.integers(1, 256, dtype=np.uint8)
        free = np.setdiff1d(np.arange(N), slots[c, :era]) if era else np.arange(N)
        p = rng.permutation(free)[:ne]
        cw[c, p] ^= rng.integers(1, 256, ne, dtype=np.uint8)
    plain, era_rows = np.arange(0, n, 2), np.arange(1, n, 2)
    # host entry points: errors only, then erasure rows
    ok, cor, d, p = m.decode_batch(cw[plain, :K], cw[plain, K:])
    ook, ocor, od, op = oracle_default.decode_batch(cw[plain, :K], cw[plain, K:])
    assert (ok == ook).all() and (cor == ocor).all() and (d == od).all() and (p == op).all()
    ok, cor, d, p = m.decode_batch(cw[era_rows, :K], cw[era_rows, K:], slots[era_rows], cnts[era_rows])
    eok, ecor, ed, ep = oracle_default.decode_batch(cw[era_rows, :K], cw[era_rows, K:],
                                                    slots[era_rows].astype(np.uint32), cnts[era_rows].astype(np.uint32))
    assert (ok == eok).all() and (cor == ecor).all() and (d == ed).all() and (p == ep).all()
    assert int(eok.sum()) == len(era_rows)
    # device entry points: handle i's shard of the rows on device 0, its own stream
    streams = [torch.cuda.Stream() for _ in range(G)]
    for rows, pos, oracle_out in ((plain, None, (ook, ocor, od, op)), (era_rows, slots, (eok, ecor, ed, ep))):
        nn = len(rows)
        shards, msgs, oks, cors, poss, cnss = [], [], [], [], [], []
        for i in range(G):
            lo, hi = P.shard_range(nn, i, G)
            shards.append(torch.from_numpy(np.ascontiguousarray(cw[rows[lo:hi]])).cuda())
            msgs.append(torch.from_numpy(np.ascontiguousarray(cw[rows[lo:hi], :K])).cuda())
            oks.append(torch.zeros(hi - lo, dtype=torch.uint8, device="cuda"))
            cors.append(torch.zeros(hi - lo, dtype=torch.uint8, device="cuda"))
            if pos is not None:
                poss.append(torch.from_numpy(np.ascontiguousarray(pos[rows[lo:hi]])).cuda())
                cnss.append(torch.from_numpy(np.ascontiguousarray(cnts[rows[lo:hi]])).cuda())
        pars = [torch.zeros((t.shape[0], NR), dtype=torch.uint8, device="cuda") for t in msgs]
        torch.cuda.synchronize()
        m.encode_batch_device([t.data_ptr() for t in msgs], K, [t.data_ptr() for t in pars], NR, K, nn,
                              [s.cuda_stream for s in streams])
        kw = {}
        if pos is not None:
            kw = dict(d_positions=[t.data_ptr() for t in poss], positions_stride=NR,
                      d_counts=[t.data_ptr() for t in cnss])
        m.decode_batch_device([t.data_ptr() for t in shards], N, [t.data_ptr() + K for t in shards], N, K, nn,
                              [o.data_ptr() for o in oks], [c.data_ptr() for c in cors],
                              streams=[s.cuda_stream for s in streams], **kw)
        torch.cuda.synchronize()
        want_par = np.concatenate([oracle_default.encode_batch(t.cpu().numpy()) for t in msgs])
        assert (np.concatenate([t.cpu().numpy() for t in pars]) == want_par).all()
        out = np.concatenate([t.cpu().numpy() for t in shards])
        w_ok, w_cor, w_d, w_p = oracle_out
        assert (np.concatenate([o.cpu().numpy() for o in oks]) == w_ok).all()
        assert (np.concatenate([c.cpu().numpy() for c in cors]) == w_cor).all()
        assert (out[:, :K] == w_d).all() and (out[:, K:] == w_p).all()
    m.close()


# ---------------------------------------------------------------------------
# compiled C drop-in programs (tests/c): the reference's README example and
# its RS codec assertions, linked against libpoporon_amd.so
# ---------------------------------------------------------------------------
def test_c_dropin_programs():
    d = os.path.join(ROOT, "tests", "c")
    r = subprocess.run([os.path.join(d, "readme_example")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Corrected 2 errors" in r.stdout and "Decoded: Hello, Reed-Solomon!" in r.stdout
    r = subprocess.run([os.path.join(d, "test_rs_api")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "all checks passed" in r.stdout


# ---------------------------------------------------------------------------
# one handle's batches beside another handle's single calls
# ---------------------------------------------------------------------------
def test_batch_beside_other_handle_single_calls(oracle_default, torch_cuda):
    """Handle B runs poporon_decode in a C loop on a host thread (the
    reference's calling pattern, SURVEY §8b: distinct handles are
    independent) while handle A encodes and decodes 2^20 codewords on the
    device.  A batch call makes B's resident server leave (ZC_YIELD) and keeps
    it from relaunching until the batch has run (api.cpp yield_servers /
    srv_launch), so A's persistent grids never wait for a CU B's server
    holds: A's results are bit-exact and A's GPU time stays within 1.2x of its
    time with B idle; every one of B's results equals the oracle's."""
    import threading

    torch = torch_cuda
    lib = P.load_library()
    A, B = P.Poporon.default(), P.Poporon.default()
    n = 1 << 20
    s = _stream(torch)
    rows = _synth(torch, n, seed=SEED + 40)
    b = rows.data_ptr()
    A.encode_batch_device(b, N, b + K, N, K, n, s)
    torch.cuda.synchronize()
    clean = rows.clone()
    clean_sum = _checksum(torch, rows)
    pos, mag = _errors(torch, n, 16, N, SEED + 41)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(n, dtype=torch.uint8, device="cuda")

    # B's codewords: 8 errors each, expected results from the oracle
    rng = np.random.default_rng(77)
    nb = 1500
    bd = rng.integers(0, 256, (nb, K), dtype=np.uint8)
    bp = oracle_default.encode_batch(bd)
    bcw = np.concatenate([bd, bp], 1)
    for c in range(nb):
        p = rng.permutation(N)[:8]
        bcw[c, p] ^= rng.integers(1, 256, 8, dtype=np.uint8)
    wok, wcor, wd, wp = oracle_default.decode_batch(bcw[:, :K], bcw[:, K:])
    stop = threading.Event()
    b_calls, b_bad = [0], [0]

    def b_loop():
        while not stop.is_set():
            d, p = bcw[:, :K].copy(), bcw[:, K:].copy()
            t, gok, gcor = T.time_decode(lib, B.h, d, p)
            assert t >= 0
            b_calls[0] += nb
            b_bad[0] += int((gok != wok).sum() + (gcor != wcor).sum() + (d != wd).any(1).sum() + (p != wp).any(1).sum())

    enc = clean.clone()  # A's encode input: the clean messages, parity rewritten in place
    eb = enc.data_ptr()

    def run_a():
        """A's encode + decode on the GPU clock; the stream is kept busy while
        the host enqueues, so host-side delays are not counted"""
        rows.copy_(clean)
        T.channel_xor(pos.data_ptr(), mag.data_ptr(), 16, b, N, n, s)
        enc[:, K:] = 0
        torch.cuda.synchronize()
        torch.cuda._sleep(2_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        A.encode_batch_device(eb, N, eb + K, N, K, n, s)
        A.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), stream=s)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def check_a():
        assert torch.equal(enc, clean)
        assert bool((ok == 1).all()) and bool((cor == 16).all())
        assert torch.equal(rows, clean)

    alone = [run_a() for _ in range(6)][1:]
    check_a()
    # B's server is resident before A's batches start
    assert B.decode(bcw[0, :K].copy(), bcw[0, K:].copy())[0] == bool(wok[0])
    th = threading.Thread(target=b_loop)
    th.start()
    try:
        import time
        time.sleep(0.05)
        beside = [run_a() for _ in range(6)][1:]
        check_a()
    finally:
        stop.set()
        th.join()
    assert b_calls[0] > 0 and b_bad[0] == 0, (b_calls[0], b_bad[0])
    ma, mb = float(np.median(alone)), float(np.median(beside))
    print(f"A alone {ma:.3f} ms, beside B's single calls {mb:.3f} ms, B calls {b_calls[0]}")
    assert mb <= 1.2 * ma, (alone, beside)
    sample = clean[::4096].cpu().numpy()
    assert (oracle_default.encode_batch(sample[:, :K]) == sample[:, K:]).all()
    assert _checksum(torch, rows) == clean_sum
