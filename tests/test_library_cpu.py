"""CPU checks of the C-ABI library (no GPU compute).

* libpoporon_amd.so loads and exports every function include/*.h declares;
* the host-side objects behave like the reference's: configs, handle getters,
  version/buildtime (tests/test_basic.c:28-36), create(NULL)/destroy(NULL)
  (tests/test_invalid.c:28-32), erasure lists (tests/test_erasure.c:30-104),
  GF handle (tests/test_gf.c:31-79), RS create (tests/test_rs.c:36-83);
* without a GPU the codec entry points fail loudly (no CPU fallback).
"""
import ctypes as C

import numpy as np
import pytest

import libpoporon_amd as P


@pytest.fixture(scope="module")
def lib():
    return P.load_library()


def test_exports_every_header_symbol(lib):
    names = P.header_symbols()
    assert len(names) >= 38
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the reference's public RS surface is all there
    for n in ("poporon_rs_config_create", "poporon_config_rs_default", "poporon_create", "poporon_destroy",
              "poporon_encode", "poporon_decode", "poporon_get_fec_type", "poporon_get_parity_size",
              "poporon_get_info_size", "poporon_get_iterations_used", "poporon_version_id", "poporon_buildtime",
              "poporon_erasure_create", "poporon_erasure_create_from_positions", "poporon_erasure_add_position",
              "poporon_erasure_reset", "poporon_erasure_destroy", "poporon_gf_create", "poporon_gf_destroy",
              "poporon_gf_mod"):
        assert n in names


def test_version_buildtime(lib, golden):
    assert lib.poporon_version_id() == int(golden["version_id"][0]) == 20000000
    assert lib.poporon_buildtime() > 0


def test_invalid_handles(lib):
    assert not lib.poporon_create(None)
    lib.poporon_destroy(None)
    assert lib.poporon_get_fec_type(None) == P.POPORON_FEC_UNKNOWN
    assert lib.poporon_get_parity_size(None) == 0
    assert lib.poporon_get_info_size(None) == 0
    assert not lib.poporon_encode(None, None, 0, None)
    assert not lib.poporon_decode(None, None, 0, None, None)


def test_out_of_scope_codecs_return_null(lib):
    assert not lib.poporon_config_ldpc_default(64, 1)
    assert not lib.poporon_config_ldpc_burst_resistant(64, 1)
    cfg = lib.poporon_config_bch_default()  # BCH is served (bch.hip)
    assert cfg
    lib.poporon_config_destroy(cfg)


def test_rs_handle_getters():
    h = P.Poporon.default()
    assert h.fec_type == P.POPORON_FEC_RS
    assert h.parity_size == 32
    assert h.info_size == 223
    assert h.lib.poporon_get_iterations_used(h.h) == 0
    assert h.supported
    h16 = P.Poporon(8, 0x11D, 1, 1, 16)
    assert h16.parity_size == 16 and h16.info_size == 239
    assert h16.supported  # general-parameter kernels (rs_generic.hip)
    assert P.Poporon(4, 0x13, 1, 2, 8).supported
    assert P.Poporon(2, 0x7, 1, 1, 2).supported
    assert not P.Poporon(1, 0x3, 1, 1, 0).supported  # GF(2): no byte-symbol RS code to serve
    with pytest.raises(P.PoporonError):
        P.Poporon(8, 0x11C, 1, 1, 32)  # non-primitive field polynomial -> NULL
    with pytest.raises(P.PoporonError):
        P.Poporon(8, 0x11D, 1, 0, 32)  # primitive_element 0 -> NULL


def test_config_destroy_after_create_keeps_handle():
    # tests/test_codec.c:30-38: the config may be destroyed right after create
    h = P.Poporon.default()
    assert h.parity_size == 32


def test_erasure_api(lib):
    e = P.Erasure(32, 8)
    for i in range(18):
        assert e.add(i)
    assert not lib.poporon_erasure_add_position(None, 0)
    e.reset()
    for i in range(5):
        assert e.add(i)
    lib.poporon_erasure_reset(None)
    e.close()
    lib.poporon_erasure_destroy(None)
    assert P.Erasure(32, 0).h
    arr = np.array([1, 3, 5, 7, 9], np.uint32)
    assert lib.poporon_erasure_create_from_positions(32, arr.ctypes.data_as(C.c_void_p), 5)
    assert not lib.poporon_erasure_create_from_positions(32, None, 5)
    assert not lib.poporon_erasure_create_from_positions(32, arr.ctypes.data_as(C.c_void_p), 0)


def test_gf_api(lib, golden):
    g = lib.poporon_gf_create(8, 0x11D)
    assert g
    for v, want in zip(golden["gf_mod_in"], golden["gf_mod_out"]):
        assert lib.poporon_gf_mod(g, int(v)) == want
    for v in range(255):
        assert lib.poporon_gf_mod(g, v) == v
    lib.poporon_gf_destroy(g)
    assert lib.poporon_gf_create(4, 0x13)
    assert not lib.poporon_gf_create(0, 0x11D)
    assert not lib.poporon_gf_create(17, 0x11D)
    lib.poporon_gf_destroy(None)


def test_rs_create_api(lib):
    for args in ((8, 0x11D, 1, 1, 16), (4, 0x13, 1, 2, 8), (8, 0x11D, 1, 1, 4), (8, 0x11D, 1, 1, 8),
                 (8, 0x11D, 1, 1, 32), (8, 0x11D, 0, 1, 16), (8, 0x11D, 2, 1, 16), (8, 0x11D, 1, 2, 16)):
        rs = lib.poporon_rs_create(*args)
        assert rs
        lib.poporon_rs_destroy(rs)
    assert not lib.poporon_rs_create(0, 0x11D, 1, 1, 16)
    lib.poporon_rs_destroy(None)


def test_no_gpu_fails_loudly():
    if P.device_count() > 0:
        pytest.skip("GPU present")
    h = P.Poporon.default()
    with pytest.raises(P.PoporonError, match="no CPU fallback"):
        h.encode(np.zeros(223, np.uint8))
    ok, n, _, _ = h.decode(np.zeros(223, np.uint8), np.zeros(32, np.uint8))
    assert not ok and n == P.DEVICE_ERROR  # a device failure, told apart from "uncorrectable" (0..32)
    assert "no CPU fallback" in P.last_error()
    with pytest.raises(P.PoporonError):
        h.encode_batch(np.zeros((4, 223), np.uint8))


def test_shard_range_partitions():
    for count in (0, 1, 7, 1 << 20, (1 << 20) + 3):
        for world in (1, 2, 3, 4, 8):
            got = [P.shard_range(count, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == count
            assert all(got[i][1] == got[i + 1][0] for i in range(world - 1))


def test_gf_mod_is_uint16_modulo():
    """rs_generic.hip computes gf_mod (src/internal/common.h:102-110) as
    (v mod 2^16) mod (2^m - 1) with a reciprocal multiply: check both claims
    for every uint16 argument and every byte symbol size."""
    v = np.arange(1 << 16, dtype=np.uint64)
    for m in range(2, 9):
        nn = (1 << m) - 1
        x = v.copy()
        while True:  # the reference's folding loop, vectorised
            big = x >= nn
            if not big.any():
                break
            y = (x[big] - nn) & 0xFFFF
            x[big] = ((y >> m) + (y & nn)) & 0xFFFF
        assert (x == v % nn).all(), m
        magic = (1 << 32) // nn + 1
        q = (v * magic) >> 32
        assert (v - q * nn == v % nn).all(), m


def test_bch_handles_and_getters():
    """BCH handles (src/poporon.c:148-170, :265-298): getters are the byte-image
    sizes of the reference (tests/golden/bch_golden.npz), invalid parameters give NULL."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "bch_golden.npz"))
    for gi, (m, poly, t) in enumerate(g["params"]):
        h = P.Bch(int(m), int(poly), int(t))
        assert h.fec_type == P.POPORON_FEC_BCH
        assert (h.parity_size, h.info_size) == tuple(int(x) for x in g[f"b{gi}_sizes"])
        assert h.lib.poporon_get_iterations_used(h.h) == 0
    d = P.Bch.default()
    assert (d.parity_size, d.info_size) == (2, 1)
    for bad in ((2, 0x7, 1), (17, 0x11D, 1), (4, 0x13, 0), (4, 0x13, 17), (4, 0x11, 2)):
        with pytest.raises(P.PoporonError):
            P.Bch(*bad)
    big = P.Bch(6, 0x43, 2)  # 63-bit codewords: created (as the reference), codec refused
    with pytest.raises(P.PoporonError, match="31 bits"):
        big.encode(np.zeros(8, np.uint8))


def test_rng_host_api_golden():
    """poporon_rng_create/next (include/poporon/rng.h) against the reference's
    own output (tests/golden/rng_golden.npz, tools/gen_golden_rng.py)."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "rng_golden.npz"))
    calls = [int(x) for x in g["calls"]]
    i = 0
    while f"seed{i}" in g.files:
        sd = bytes(g[f"seed{i}"])
        r = P.Rng(sd if sd else None)
        got = np.concatenate([r.next(n) for n in calls])
        assert (got == g[f"stream{i}"]).all(), i
        i += 1
    lib = P.load_library()
    assert not lib.poporon_rng_next(None, None, 4)
    r = P.Rng(1)
    assert not lib.poporon_rng_next(r.h, None, 4)
    buf = np.zeros(4, np.uint8)
    assert not lib.poporon_rng_next(r.h, buf.ctypes.data_as(C.c_void_p), 0)
    lib.poporon_rng_destroy(None)


def test_c_dropin_builds_and_checks_arguments():
    """tests/c/test_rs_api.c compiles against include/poporon.h alone, links
    libpoporon_amd.so and passes the reference's argument checks
    (tests/test_codec.c:69-71, :220-223) without a GPU."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "tests", "c")])
    r = subprocess.run([os.path.join(root, "tests", "c", "test_rs_api"), "--no-gpu"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


def test_multi_partition_and_argument_checks(lib):
    first, n = C.c_size_t(0), C.c_size_t(0)
    for count in (0, 5, 1000, (1 << 26) + 7):
        for parts in (1, 2, 3, 8):
            spans = []
            for p in range(parts):
                assert lib.poporon_amd_multi_range(count, parts, p, C.byref(first), C.byref(n))
                spans.append((first.value, first.value + n.value))
            assert spans[0][0] == 0 and spans[-1][1] == count
            assert all(spans[i][1] == spans[i + 1][0] for i in range(parts - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
    assert not lib.poporon_amd_multi_range(10, 0, 0, C.byref(first), C.byref(n))
    assert not lib.poporon_amd_multi_range(10, 2, 2, C.byref(first), C.byref(n))
    assert lib.poporon_amd_multi_device_count(None) == 0
    assert not lib.poporon_amd_multi_handle(None, 0)
    lib.poporon_amd_multi_destroy(None)
    assert not lib.poporon_encode_batch_multi(None, None, 0, None, 0, 223, 1)
    if P.device_count() == 0:
        cfg = lib.poporon_config_rs_default()
        assert not lib.poporon_amd_multi_create(cfg, None, 0)  # no device: NULL, with a message
        assert "no HIP device" in P.last_error()
        lib.poporon_config_destroy(cfg)


def test_syndrome_api_argument_checks(lib):
    h = P.Poporon.default()
    assert not lib.poporon_syndrome_batch_device(h.h, None, 255, None, 255, 223, 4, None, 32, None, None)
    assert not lib.poporon_syndrome_batch_device(None, None, 255, None, 255, 223, 0, None, 32, None, None)
    b = P.Bch.default()
    x = np.zeros(64, np.uint8)
    xp = x.ctypes.data_as(C.c_void_p)
    assert not lib.poporon_syndrome_batch_device(b.h, xp, 3, xp, 3, 1, 1, xp, 32, None, None)
    assert "RS handles" in P.last_error()
