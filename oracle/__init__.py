"""CPU oracle for the RS(255,223) hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker (or the timed CPU
baseline).  The product, ``libpoporon_amd``, never imports it.

Two CPU implementations are reachable from here:

* ``Oracle``    -- ctypes binding of ``oracle/liboracle.so``, the clean-room C
  restatement in ``oracle/rs_oracle.c`` (pinned against ``tests/golden``).
* ``Reference`` -- ctypes binding of ``oracle/_ref/libpoporon_ref.so``, the real
  libpoporon compiled from ``/root/reference/src`` by ``oracle/Makefile``.  Only
  present where it was built (this container; it travels to the GPU box as a
  built artefact).  Driven through the reference's public C API only, except
  for ``rs_tables``/``last_syndrome`` which mirror its internal structs to read
  the GF tables, the generator and the handle's syndrome scratch.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpoporon_ref.so")
REF_AVX2_SO = os.path.join(HERE, "_ref", "libpoporon_ref_avx2.so")

_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)


def _ptr(a, t=_u8p):
    return a.ctypes.data_as(t) if a is not None else None


class Oracle:
    """Clean-room restatement (oracle/rs_oracle.c)."""

    def __init__(self, m=8, gfpoly=0x11D, fcr=1, prim=1, nroots=32, so=ORACLE_SO):
        self.lib = C.CDLL(so)
        L = self.lib
        L.oracle_rs_sizeof.restype = C.c_size_t
        L.oracle_rs_init.argtypes = [C.c_void_p, C.c_uint8, C.c_uint16, C.c_uint16, C.c_uint16, C.c_uint16]
        L.oracle_gf_mod.argtypes = [C.c_void_p, C.c_uint32]
        L.oracle_gf_mod.restype = C.c_uint16
        L.oracle_rs_encode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p]
        L.oracle_rs_syndrome.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, _u16p]
        L.oracle_rs_decode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, C.c_int, _u32p, C.c_uint32, _u16p,
                                       C.POINTER(C.c_size_t)]
        L.oracle_rs_encode_batch.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, C.c_size_t, C.c_size_t, C.c_size_t]
        L.oracle_rs_decode_batch.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, C.c_size_t, C.c_size_t, C.c_size_t,
                                             C.c_int, _u32p, C.c_size_t, _u32p, _u8p, _u32p]
        L.oracle_rs_encode_batch_mt.argtypes = L.oracle_rs_encode_batch.argtypes + [C.c_int]
        L.oracle_rs_decode_batch_mt.argtypes = L.oracle_rs_decode_batch.argtypes + [C.c_int]
        self._buf = C.create_string_buffer(L.oracle_rs_sizeof())
        self.h = C.cast(self._buf, C.c_void_p)
        if L.oracle_rs_init(self.h, m, gfpoly, fcr, prim, nroots) != 0:
            raise ValueError("oracle_rs_init rejected the parameters")
        self.m, self.nroots, self.fcr, self.prim = m, nroots, fcr, prim
        self.nn = (1 << m) - 1

    # -- tables -----------------------------------------------------------------
    def tables(self):
        """(alog, log, genpoly_log) as numpy arrays (field-sized / nroots+1)."""
        # struct layout: u8 m; u16 nn, gfpoly, fcr, prim, nroots, iprim; u16 alog[65536]; u16 log[65536]; u16 gen[256]
        raw = np.frombuffer(self._buf, dtype=np.uint8)
        off = 2 + 2 * 6
        alog = raw[off:off + 2 * 65536].view(np.uint16)[: self.nn + 1].copy()
        off += 2 * 65536
        log = raw[off:off + 2 * 65536].view(np.uint16)[: self.nn + 1].copy()
        off += 2 * 65536
        gen = raw[off:off + 2 * 256].view(np.uint16)[: self.nroots + 1].copy()
        return alog, log, gen

    def gf_mod(self, v):
        return self.lib.oracle_gf_mod(self.h, v)

    # -- single codeword --------------------------------------------------------
    def encode(self, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        par = np.zeros(self.nroots, np.uint8)
        self.lib.oracle_rs_encode(self.h, _ptr(data), data.size, _ptr(par))
        return par

    def syndrome(self, data, parity):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        parity = np.ascontiguousarray(parity, dtype=np.uint8)
        s = np.zeros(self.nroots, np.uint16)
        flag = self.lib.oracle_rs_syndrome(self.h, _ptr(data), data.size, _ptr(parity), _ptr(s, _u16p))
        return bool(flag), s

    def decode(self, data, parity, erasures=None, ext_syn=None, eras_mode=None):
        """In-place on copies; returns (ok, corrected, data, parity)."""
        d = np.array(data, dtype=np.uint8, copy=True)
        p = np.array(parity, dtype=np.uint8, copy=True)
        n = C.c_size_t(0)
        if eras_mode is None:
            eras_mode = erasures is not None
        if erasures is not None:
            e = np.asarray(erasures, dtype=np.uint32)
            cnt = e.size
            pos = np.zeros(max(cnt, self.nroots), np.uint32)
            pos[:cnt] = e
        else:
            cnt, pos = 0, np.zeros(self.nroots, np.uint32)
        syn = None if ext_syn is None else np.ascontiguousarray(ext_syn, dtype=np.uint16)
        ok = self.lib.oracle_rs_decode(self.h, _ptr(d), d.size, _ptr(p), int(bool(eras_mode)), _ptr(pos, _u32p), cnt,
                                       _ptr(syn, _u16p), C.byref(n))
        return bool(ok), int(n.value), d, p

    # -- batches ----------------------------------------------------------------
    def encode_batch(self, data, threads=0):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        count, size = data.shape
        par = np.zeros((count, self.nroots), np.uint8)
        if threads:
            self.lib.oracle_rs_encode_batch_mt(self.h, _ptr(data), size, _ptr(par), self.nroots, size, count, threads)
        else:
            self.lib.oracle_rs_encode_batch(self.h, _ptr(data), size, _ptr(par), self.nroots, size, count)
        return par

    def decode_batch(self, data, parity, erasures=None, counts=None, threads=0):
        """data (count,size), parity (count,nroots); erasures (count, >=nroots) uint32 slots + counts.
        Returns (ok u8[count], corrected u32[count], data', parity')."""
        d = np.array(data, dtype=np.uint8, copy=True, order="C")
        p = np.array(parity, dtype=np.uint8, copy=True, order="C")
        count, size = d.shape
        ok = np.zeros(count, np.uint8)
        cor = np.zeros(count, np.uint32)
        if erasures is not None:
            e = np.ascontiguousarray(erasures, dtype=np.uint32)
            cn = np.ascontiguousarray(counts, dtype=np.uint32)
            args = (1, _ptr(e, _u32p), e.shape[1], _ptr(cn, _u32p))
        else:
            args = (0, None, 0, None)
        if threads:
            self.lib.oracle_rs_decode_batch_mt(self.h, _ptr(d), size, _ptr(p), p.shape[1], size, count, *args,
                                               _ptr(ok), _ptr(cor, _u32p), threads)
        else:
            self.lib.oracle_rs_decode_batch(self.h, _ptr(d), size, _ptr(p), p.shape[1], size, count, *args, _ptr(ok),
                                            _ptr(cor, _u32p))
        return ok, cor, d, p


# -----------------------------------------------------------------------------
# The real reference, driven through its own C API
# -----------------------------------------------------------------------------
class _RefGF(C.Structure):  # src/internal/common.h:46-52
    _fields_ = [("symbol_size", C.c_uint8), ("field_size", C.c_uint8), ("log2exp", _u16p), ("exp2log", _u16p),
                ("generator_polynomial", C.c_uint16)]


class _RefRS(C.Structure):  # src/internal/common.h:54-60
    _fields_ = [("gf", C.POINTER(_RefGF)), ("first_consecutive_root", C.c_uint16), ("primitive_element", C.c_uint16),
                ("num_roots", C.c_uint16), ("generator_polynomial", _u16p)]


class _RefBuf(C.Structure):  # src/internal/common.h:62-72
    _fields_ = [("error_locator", _u16p), ("syndrome", _u16p), ("coefficients", _u16p), ("polynomial", _u16p),
                ("error_evaluator", _u16p), ("error_roots", _u16p), ("register_coefficients", _u16p),
                ("error_locations", _u16p), ("primitive_inverse", C.c_uint16)]


class _RefHandleRS(C.Structure):  # src/internal/common.h:74-100 (fec_type + ctx.rs)
    _fields_ = [("fec_type", C.c_int), ("rs", C.POINTER(_RefRS)), ("buffer", C.POINTER(_RefBuf)),
                ("erasure", C.c_void_p), ("ext_syndrome", _u16p), ("last_corrected", C.c_size_t)]


def reference_available(so=REF_SO):
    return os.path.exists(so)


class Reference:
    """libpoporon itself (oracle/_ref), one handle per instance."""

    def __init__(self, m=8, gfpoly=0x11D, fcr=1, prim=1, nroots=32, erasure=False, ext_syn=None, so=REF_SO,
                 erasure_capacity=None):
        L = self.lib = C.CDLL(so)
        L.poporon_rs_config_create.restype = C.c_void_p
        L.poporon_rs_config_create.argtypes = [C.c_uint8, C.c_uint16, C.c_uint16, C.c_uint16, C.c_uint8, C.c_void_p,
                                               _u16p]
        L.poporon_create.restype = C.c_void_p
        L.poporon_create.argtypes = [C.c_void_p]
        L.poporon_destroy.argtypes = [C.c_void_p]
        L.poporon_config_destroy.argtypes = [C.c_void_p]
        L.poporon_encode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p]
        L.poporon_encode.restype = C.c_bool
        L.poporon_decode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]
        L.poporon_decode.restype = C.c_bool
        L.poporon_erasure_create.restype = C.c_void_p
        L.poporon_erasure_create.argtypes = [C.c_uint16, C.c_uint32]
        L.poporon_erasure_add_position.argtypes = [C.c_void_p, C.c_uint32]
        L.poporon_erasure_add_position.restype = C.c_bool
        L.poporon_erasure_reset.argtypes = [C.c_void_p]
        L.poporon_erasure_destroy.argtypes = [C.c_void_p]
        L.poporon_gf_create.restype = C.c_void_p
        L.poporon_gf_create.argtypes = [C.c_uint8, C.c_uint16]
        L.poporon_gf_mod.argtypes = [C.c_void_p, C.c_uint16]
        L.poporon_gf_mod.restype = C.c_uint8
        L.poporon_gf_destroy.argtypes = [C.c_void_p]
        L.poporon_rs_create.restype = C.c_void_p
        L.poporon_rs_create.argtypes = [C.c_uint8, C.c_uint16, C.c_uint16, C.c_uint16, C.c_uint8]
        L.poporon_rs_destroy.argtypes = [C.c_void_p]
        L.poporon_version_id.restype = C.c_uint32
        L.poporon_buildtime.restype = C.c_uint32
        self.nroots = nroots
        self.eras = L.poporon_erasure_create(nroots, erasure_capacity or nroots) if erasure else None
        self._syn = None
        if ext_syn is not None:
            self._syn = (C.c_uint16 * nroots)(*[int(x) for x in ext_syn])
        cfg = L.poporon_rs_config_create(m, gfpoly, fcr, prim, nroots, self.eras,
                                         C.cast(self._syn, _u16p) if self._syn is not None else None)
        self.h = L.poporon_create(cfg)
        L.poporon_config_destroy(cfg)
        if not self.h:
            raise ValueError("poporon_create returned NULL")

    def close(self):
        if self.h:
            self.lib.poporon_destroy(self.h)
            self.h = None
        if self.eras:
            self.lib.poporon_erasure_destroy(self.eras)
            self.eras = None

    __del__ = close

    def set_erasures(self, positions):
        self.lib.poporon_erasure_reset(self.eras)
        for p in positions:
            self.lib.poporon_erasure_add_position(self.eras, int(p))

    def encode(self, data):
        d = np.array(data, dtype=np.uint8, copy=True)
        par = np.zeros(self.nroots, np.uint8)
        ok = self.lib.poporon_encode(self.h, _ptr(d), d.size, _ptr(par))
        return bool(ok), par

    def decode(self, data, parity):
        d = np.array(data, dtype=np.uint8, copy=True)
        p = np.array(parity, dtype=np.uint8, copy=True)
        n = C.c_size_t(0)
        ok = self.lib.poporon_decode(self.h, _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8)), d.size, _ptr(p),
                                     C.byref(n))
        return bool(ok), int(n.value), d, p

    def last_syndrome(self):
        h = C.cast(self.h, C.POINTER(_RefHandleRS)).contents
        s = h.buffer.contents.syndrome
        return np.array([s[i] for i in range(self.nroots)], np.uint16)

    def rs_tables(self):
        h = C.cast(self.h, C.POINTER(_RefHandleRS)).contents
        rs = h.rs.contents
        gf = rs.gf.contents
        nn = gf.field_size
        alog = np.array([gf.log2exp[i] for i in range(nn + 1)], np.uint16)
        log = np.array([gf.exp2log[i] for i in range(nn + 1)], np.uint16)
        gen = np.array([rs.generator_polynomial[i] for i in range(rs.num_roots + 1)], np.uint16)
        return alog, log, gen, h.buffer.contents.primitive_inverse


# -----------------------------------------------------------------------------
# binary BCH (oracle/bch_oracle.c) and the reference's BCH handle
# -----------------------------------------------------------------------------
class BchOracle:
    """Clean-room restatement of the reference's BCH codec (oracle/bch_oracle.c)."""

    def __init__(self, m=4, poly=0x13, t=3, so=ORACLE_SO):
        L = self.lib = C.CDLL(so)
        L.oracle_bch_sizeof.restype = C.c_size_t
        L.oracle_bch_init.argtypes = [C.c_void_p, C.c_uint8, C.c_uint16, C.c_uint8]
        L.oracle_bch_data_bits.argtypes = L.oracle_bch_parity_bits.argtypes = [C.c_void_p]
        L.oracle_bch_data_bits.restype = L.oracle_bch_parity_bits.restype = C.c_uint32
        L.oracle_bch_encode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p]
        L.oracle_bch_decode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]
        self._buf = C.create_string_buffer(L.oracle_bch_sizeof())
        self.h = C.cast(self._buf, C.c_void_p)
        rc = L.oracle_bch_init(self.h, m, poly, t)
        if rc != 0:
            raise ValueError(f"oracle_bch_init: {rc}")
        self.k = L.oracle_bch_data_bits(self.h)
        self.pbits = L.oracle_bch_parity_bits(self.h)
        self.data_bytes = (self.k + 7) // 8
        self.parity_bytes = (self.pbits + 7) // 8

    def encode(self, data):
        d = np.ascontiguousarray(data, dtype=np.uint8)
        par = np.zeros(max(1, self.parity_bytes), np.uint8)
        ok = self.lib.oracle_bch_encode(self.h, _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8)), d.size,
                                        _ptr(par))
        return bool(ok), par[: self.parity_bytes]

    def decode(self, data, parity, corrected_init=0):
        d = np.array(data, dtype=np.uint8, copy=True)
        p = np.ascontiguousarray(parity, dtype=np.uint8)
        n = C.c_size_t(corrected_init)
        ok = self.lib.oracle_bch_decode(self.h, _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8)), d.size,
                                        _ptr(p) if p.size else _ptr(np.zeros(1, np.uint8)), C.byref(n))
        return bool(ok), int(n.value), d


class ReferenceBch:
    """libpoporon's BCH handle (oracle/_ref), driven through poporon_encode/decode."""

    def __init__(self, m=4, poly=0x13, t=3, so=REF_SO):
        L = self.lib = C.CDLL(so)
        L.poporon_bch_config_create.restype = C.c_void_p
        L.poporon_bch_config_create.argtypes = [C.c_uint8, C.c_uint16, C.c_uint8]
        L.poporon_create.restype = C.c_void_p
        L.poporon_create.argtypes = [C.c_void_p]
        L.poporon_destroy.argtypes = [C.c_void_p]
        L.poporon_config_destroy.argtypes = [C.c_void_p]
        L.poporon_encode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p]
        L.poporon_encode.restype = C.c_bool
        L.poporon_decode.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]
        L.poporon_decode.restype = C.c_bool
        L.poporon_get_parity_size.argtypes = L.poporon_get_info_size.argtypes = [C.c_void_p]
        L.poporon_get_parity_size.restype = L.poporon_get_info_size.restype = C.c_size_t
        cfg = L.poporon_bch_config_create(m, poly, t)
        self.h = L.poporon_create(cfg)
        L.poporon_config_destroy(cfg)
        if not self.h:
            raise ValueError("poporon_create returned NULL")
        self.parity_bytes = L.poporon_get_parity_size(self.h)
        self.info_bytes = L.poporon_get_info_size(self.h)

    def close(self):
        if self.h:
            self.lib.poporon_destroy(self.h)
            self.h = None

    __del__ = close

    def encode(self, data):
        d = np.array(data, dtype=np.uint8, copy=True)
        par = np.zeros(max(1, self.parity_bytes), np.uint8)
        ok = self.lib.poporon_encode(self.h, _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8)), d.size, _ptr(par))
        return bool(ok), par[: self.parity_bytes]

    def decode(self, data, parity, corrected_init=0):
        d = np.array(data, dtype=np.uint8, copy=True)
        p = np.array(parity, dtype=np.uint8, copy=True)
        n = C.c_size_t(corrected_init)
        ok = self.lib.poporon_decode(self.h, _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8)), d.size,
                                     _ptr(p) if p.size else _ptr(np.zeros(1, np.uint8)), C.byref(n))
        return bool(ok), int(n.value), d
