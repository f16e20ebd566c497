"""bench.py's parity sample checker, on CPU.

The bench compares every 4096th codeword of each timed mode with the
reference CPU path after its timed loops.  These tests pin the checker
itself: it accepts the reference's own results, flags any changed byte, ok
or corrected_num, and its two kinds -- the reference library driven through
its public API (erasure lists refilled per codeword so the slots past the
count are the row's stale entries, quirks Q1/Q2) and the restatement's batch
call -- agree on erasure and errata samples.
"""
import numpy as np
import pytest

import bench
from oracle import Oracle, reference_available

K, NR = 223, 32


def _errata_sample(rng, n, ne, nerr):
    o = Oracle()
    data = rng.integers(0, 256, (n, K), dtype=np.uint8)
    cw = np.concatenate([data, o.encode_batch(data)], 1)
    # stale slots inside the message: the reference writes data[slot] for a
    # slot >= size past the caller's buffer (quirk Q4, undefined there)
    slots = rng.integers(0, K, (n, NR)).astype(np.uint8)
    cnt = np.full(n, ne, np.uint8)
    for c in range(n):
        er = rng.permutation(K)[:ne]  # insertion order: Q1
        slots[c, :ne] = er
        cw[c, er] ^= rng.integers(1, 256, ne, dtype=np.uint8)
        rest = np.setdiff1d(np.arange(255), er)
        x = rng.permutation(rest)[:nerr]
        cw[c, x] ^= rng.integers(1, 256, nerr, dtype=np.uint8)
    ok, cor, d, p = o.decode_batch(cw[:, :K], cw[:, K:], slots.astype(np.uint32), cnt.astype(np.uint32))
    return {"in": cw, "out": np.concatenate([d, p], 1), "ok": ok, "cor": cor.astype(np.uint8), "slots": slots,
            "cnt": cnt}


@pytest.fixture(params=["reference", "port"])
def checker(request, monkeypatch):
    if request.param == "reference" and not reference_available():
        pytest.skip("oracle/_ref not built (no /root/reference)")
    if request.param == "port":
        monkeypatch.setattr("oracle.reference_available", lambda *a, **k: False)
    chk = bench.ParityChecker()
    assert chk.kind == request.param
    return chk


@pytest.mark.parametrize("ne,nerr", [(32, 0), (16, 8), (20, 0), (8, 6)])
def test_checker_accepts_oracle_erasure_results(checker, ne, nerr):
    sm = _errata_sample(np.random.default_rng(ne * 7 + nerr), 40, ne, nerr)
    assert checker.check(sm) == 0


def test_checker_flags_any_difference(checker):
    sm = _errata_sample(np.random.default_rng(3), 30, 16, 8)
    for field, c in (("out", 2), ("ok", 5), ("cor", 7)):
        bad = {k: v.copy() for k, v in sm.items()}
        if field == "out":
            bad["out"][c, 100] ^= 1
        else:
            bad[field][c] ^= 1
        assert checker.check(bad) == 1, field


def test_checker_encode_and_errors(checker):
    import testutil as T
    o = Oracle()
    msgs = T.synth_rows_cpu(bench.SEED, 0, 24, K)
    par = o.encode_batch(msgs)
    assert checker.check({"msg": msgs, "got_par": par}) == 0
    par[3, 0] ^= 0x80
    assert checker.check({"msg": msgs, "got_par": par}) == 1
    pos, mag = T.synth_errors_cpu(bench.SEED + 1, 0, 24, 20, 255)  # beyond t: failures, miscorrections
    rows = bench.channel_rows(np.concatenate([msgs, o.encode_batch(msgs)], 1), pos, mag)
    ok, cor, d, p = o.decode_batch(rows[:, :K], rows[:, K:])
    sm = {"in": rows, "out": np.concatenate([d, p], 1), "ok": ok, "cor": cor.astype(np.uint8)}
    assert checker.check(sm) == 0


def test_mixed_counts_deterministic_and_sharded():
    a = bench.mixed_counts(0, 4096)
    b = np.concatenate([bench.mixed_counts(0, 1000), bench.mixed_counts(1000, 3096)])
    assert (a == b).all()
    assert a.max() <= bench.MIXED_CAP
    past = (a > 16).mean()
    assert 0.03 < past < 0.10 and 10 < a.mean() < 13
