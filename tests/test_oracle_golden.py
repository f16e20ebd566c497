"""Pin the CPU restatement (oracle/rs_oracle.c) to the reference's golden vectors.

tests/golden/rs255_golden.npz was produced by tools/gen_golden.py from the real
libpoporon (oracle/_ref).  Every class of SURVEY.md 8(c) is covered: GF tables,
generator, gf_mod, encode (full and shortened), syndromes, decode with 0..25
errors over data and parity, constructed miscorrections, erasures sorted /
unsorted (Q1), erasures + errors (Q2), e = 0 erasure mode (Q3), external
syndromes and invalid sizes.  Bit-exact: bytes, bool and corrected_num.
"""
import numpy as np
import pytest

from oracle import Oracle, Reference, reference_available

NR = 32


def test_appendix_b_known_answers(oracle_default):
    o = oracle_default
    alog, log, gen = o.tables()
    assert list(alog[:16]) == [1, 2, 4, 8, 16, 32, 64, 128, 29, 58, 116, 232, 205, 135, 19, 38]
    assert alog[255] == 0
    assert list(log[:16]) == [255, 0, 1, 25, 2, 50, 26, 198, 3, 223, 51, 238, 27, 104, 199, 75]
    assert list(gen) == [18, 251, 215, 28, 80, 107, 248, 53, 84, 194, 91, 59, 176, 99, 203, 137, 43, 104, 137, 0,
                         44, 149, 148, 218, 75, 11, 173, 254, 194, 109, 8, 11, 0]
    d = np.arange(223, dtype=np.uint8)
    assert o.encode(d).tobytes().hex() == "66d474a49f3de52711f4f543fd129cd973491fae1b8c459f68dbfebbada90a74"
    z = np.zeros(223, np.uint8)
    z[222] = 1
    assert o.encode(z).tobytes().hex() == "e81dbd328ef6e80f2b52a4ee019e0d779ee086e3d2a3326b281b68fd18efd82d"
    z[:] = 0
    z[0] = 1
    assert o.encode(z).tobytes().hex() == "8b1be9a3e3cb721bba1c2e5c068b93b1039337e7b7d4cae3619cf4e1de748df3"
    assert not o.encode(np.zeros(223, np.uint8)).any()
    cw = np.concatenate([d, o.encode(d)])
    cw[0] ^= 1
    cw[100] ^= 0x80
    flag, s = o.syndrome(cw[:223], cw[223:])
    assert flag
    assert list(s) == [64, 88, 143, 118, 63, 223, 188, 157, 3, 94, 152, 47, 209, 32, 164, 231, 2, 174, 34, 81, 73,
                       199, 27, 17, 58, 52, 235, 99, 58, 186, 206, 85]
    ok, n, od, op = o.decode(cw[:223], cw[223:])
    assert ok and n == 2 and (od == d).all()


@pytest.mark.parametrize("i", range(8))
def test_tables_generator_iprim(golden, i):
    m, poly, fcr, prim, nr = (int(x) for x in golden["param_sets"][i])
    o = Oracle(m, poly, fcr, prim, nr)
    alog, log, gen = o.tables()
    assert (alog == golden[f"p{i}_alog"]).all()
    assert (log == golden[f"p{i}_log"]).all()
    assert (gen == golden[f"p{i}_gen"]).all()
    assert o.lib.oracle_rs_init  # handle alive
    # primitive inverse is internal; re-derive through the Chien mapping below via decode tests


def test_gf_mod(golden, oracle_default):
    for v, want in zip(golden["gf_mod_in"], golden["gf_mod_out"]):
        assert oracle_default.gf_mod(int(v)) == want
    for v in range(65536):
        assert oracle_default.gf_mod(v) == v % 255


def test_encode_golden(golden, oracle_default):
    for s, d, p in zip(golden["enc_size"], golden["enc_data"], golden["enc_parity"]):
        assert (oracle_default.encode(d[:s]) == p).all()


def test_syndrome_golden(golden, oracle_default):
    for s, inp, syn in zip(golden["dec_size"], golden["dec_in"], golden["dec_syn"]):
        L = int(s) + NR
        _, got = oracle_default.syndrome(inp[:s], inp[s:L])
        assert (got == syn).all()


def test_decode_golden(golden, oracle_default):
    for s, inp, ok, cor, out in zip(golden["dec_size"], golden["dec_in"], golden["dec_ok"], golden["dec_cor"],
                                    golden["dec_out"]):
        L = int(s) + NR
        g_ok, g_n, od, op = oracle_default.decode(inp[:s], inp[s:L])
        assert g_ok == bool(ok) and g_n == cor
        assert (np.concatenate([od, op]) == out[:L]).all()


def test_decode_golden_batch(golden, oracle_default):
    sel = golden["dec_size"] == 223
    ok, cor, d, p = oracle_default.decode_batch(golden["dec_in"][sel, :223], golden["dec_in"][sel, 223:])
    assert (ok == golden["dec_ok"][sel]).all() and (cor == golden["dec_cor"][sel]).all()
    assert (np.concatenate([d, p], 1) == golden["dec_out"][sel]).all()


def test_erasure_golden(golden, oracle_default):
    for s, slots, e, inp, ok, cor, out in zip(golden["era_size"], golden["era_slots"], golden["era_count"],
                                              golden["era_in"], golden["era_ok"], golden["era_cor"], golden["era_out"]):
        L = int(s) + NR
        o = oracle_default
        import ctypes as C
        d = inp[:s].copy()
        p = inp[s:L].copy()
        n = C.c_size_t(0)
        from oracle import _ptr, _u32p
        g_ok = o.lib.oracle_rs_decode(o.h, _ptr(d), int(s), _ptr(p), 1, _ptr(np.ascontiguousarray(slots), _u32p),
                                      int(e), None, C.byref(n))
        assert bool(g_ok) == bool(ok) and n.value == cor
        assert (np.concatenate([d, p]) == out[:L]).all()


def test_ext_syndrome_golden(golden, oracle_default):
    for inp, syn, ok, cor, out in zip(golden["xs_in"], golden["xs_syn"], golden["xs_ok"], golden["xs_cor"],
                                      golden["xs_out"]):
        g_ok, g_n, od, op = oracle_default.decode(inp[:223], inp[223:], ext_syn=syn)
        assert g_ok == bool(ok) and g_n == cor and (np.concatenate([od, op]) == out).all()


def test_invalid_sizes(golden, oracle_default):
    for size, ok, cor in golden["invalid"]:
        d = np.zeros(max(int(size), 1), np.uint8)
        g_ok, g_n, _, _ = oracle_default.decode(d[: int(size)], np.zeros(NR, np.uint8))
        assert g_ok == bool(ok) and g_n == cor


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built here")
def test_restatement_vs_reference_random():
    """Direct cross-check against the compiled reference (where it exists)."""
    o, r = Oracle(), Reference()
    rng = np.random.default_rng(7)
    for _ in range(600):
        size = int(rng.integers(1, 224))
        d = rng.integers(0, 256, size, dtype=np.uint8)
        p = o.encode(d)
        assert (p == r.encode(d)[1]).all()
        ne = int(rng.integers(0, 22))
        cw = np.concatenate([d, p])
        pos = rng.permutation(size + NR)[:ne]
        cw[pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
        a, b = o.decode(cw[:size], cw[size:]), r.decode(cw[:size], cw[size:])
        assert a[0] == b[0] and a[1] == b[1] and (a[2] == b[2]).all() and (a[3] == b[3]).all()


# ---------------------------------------------------------------------------
# general parameters (tests/golden/rs_params_golden.npz, tools/gen_golden_params.py)
# ---------------------------------------------------------------------------
PARAMS_GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "rs_params_golden.npz")


@pytest.fixture(scope="module")
def pgolden():
    return np.load(PARAMS_GOLDEN)


@pytest.mark.parametrize("gi", range(13))
def test_oracle_general_parameters_golden(pgolden, gi):
    m, poly, fcr, prim, nr = (int(x) for x in pgolden["params"][gi])
    o = Oracle(m, poly, fcr, prim, nr)
    g = lambda k: pgolden[f"g{gi}_{k}"]  # noqa: E731
    for s, d, p in zip(g("enc_size"), g("enc_data"), g("enc_parity")):
        assert (o.encode(d[:s]) == p).all()
    for s, inp, out, ok, cor in zip(g("dec_size"), g("dec_in"), g("dec_out"), g("dec_ok"), g("dec_cor")):
        s = int(s)
        gok, gn, gd, gp = o.decode(inp[:s], inp[s:s + nr])
        assert gok == bool(ok) and gn == cor and (np.concatenate([gd, gp]) == out[:s + nr]).all()
    for s, e, slots, inp, out, ok, cor in zip(g("era_size"), g("era_count"), g("era_slots"), g("era_in"),
                                              g("era_out"), g("era_ok"), g("era_cor")):
        s, e = int(s), int(e)
        gok, gn, gd, gp = o.decode(inp[:s], inp[s:s + nr], erasures=slots[:e])
        assert gok == bool(ok) and gn == cor and (np.concatenate([gd, gp]) == out[:s + nr]).all()
    k = (1 << m) - 1 - nr
    for syn, inp, out, ok, cor in zip(g("xs_syn"), g("xs_in"), g("xs_out"), g("xs_ok"), g("xs_cor")):
        gok, gn, gd, gp = o.decode(inp[:k], inp[k:k + nr], ext_syn=syn)
        assert gok == bool(ok) and gn == cor and (np.concatenate([gd, gp]) == out[:k + nr]).all()


# ---------------------------------------------------------------------------
# binary BCH (tests/golden/bch_golden.npz, tools/gen_golden_bch.py)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def bgolden():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "bch_golden.npz"))


@pytest.mark.parametrize("gi", range(12))
def test_bch_oracle_golden(bgolden, gi):
    from oracle import BchOracle
    m, poly, t = (int(x) for x in bgolden["params"][gi])
    o = BchOracle(m, poly, t)
    g = lambda k: bgolden[f"b{gi}_{k}"]  # noqa: E731
    pb, ib = (int(x) for x in g("sizes"))
    assert (o.parity_bytes, o.data_bytes) == (pb, ib)
    for d, p in zip(g("enc_data"), g("enc_parity")):
        ok, par = o.encode(d[:ib])
        assert ok and (par == p[:pb]).all()
    for d, p, out, ok, cor in zip(g("dec_data"), g("dec_parity"), g("dec_out"), g("dec_ok"), g("dec_cor")):
        gok, gn, gd = o.decode(d[:ib], p[:pb], 777)  # 777: left untouched on failure, as the reference
        assert gok == bool(ok) and gn == cor and (gd == out[:ib]).all()


def test_bch_oracle_vs_reference_random():
    if not reference_available():
        pytest.skip("oracle/_ref not built")
    from oracle import BchOracle, ReferenceBch
    rng = np.random.default_rng(5)
    for m, poly, t in ((4, 0x13, 3), (5, 0x25, 3), (5, 0x25, 6), (3, 0x0B, 1)):
        o, r = BchOracle(m, poly, t), ReferenceBch(m, poly, t)
        ib, pb = o.data_bytes, o.parity_bytes
        for _ in range(3000):
            d = rng.integers(0, 256, ib, dtype=np.uint8)
            p = rng.integers(0, 256, pb, dtype=np.uint8)
            assert (o.encode(d)[1] == r.encode(d)[1]).all()
            a, b = o.decode(d, p, 5), r.decode(d, p, 5)
            assert a[0] == b[0] and a[1] == b[1] and (a[2] == b[2]).all()
