"""libpoporon_amd -- MI355X-native Reed-Solomon engine behind libpoporon's C API.

The product is the C-ABI shared library ``libpoporon_amd/libpoporon_amd.so``
(headers in ``include/``): the reference's ``poporon_*`` entry points
(include/poporon.h:67-99 of colopl/libpoporon) served by HIP kernels for
gfx950, plus the batch / device-pointer extension of ``include/poporon_amd.h``.

This module is the host-side mirror used by Python callers, the tests and
``bench.py``: a thin ctypes binding whose names, argument meaning and error
behaviour follow the reference API (``poporon_create``, ``poporon_encode``,
``poporon_decode``, erasure lists ...).  It never computes RS arithmetic
itself and it never falls back to a CPU path: if the shared library is
missing, importing the binding raises; if no GPU is usable, the codec calls
fail with the library's error message.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("POPORON_AMD_LIB") or os.path.join(HERE, "libpoporon_amd.so")  # override: experiments
INCLUDE_DIR = os.path.join(ROOT, "include")

POPORON_FEC_RS = 1
POPORON_FEC_LDPC = 2
POPORON_FEC_BCH = 3
POPORON_FEC_UNKNOWN = 255
# poporon_decode's *corrected_num after a device-side failure (include/poporon_amd.h)
DEVICE_ERROR = (1 << 64) - 1

_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)
_vp = C.c_void_p

# name: (restype, argtypes)
_SIGS = {
    "poporon_rs_config_create": (_vp, [C.c_uint8, C.c_uint16, C.c_uint16, C.c_uint16, C.c_uint8, _vp, _vp]),
    "poporon_ldpc_config_create": (_vp, [C.c_size_t, C.c_int, C.c_int, C.c_uint32, C.c_bool, C.c_bool, C.c_bool,
                                         C.c_uint32, C.c_uint32, C.c_uint32, _vp, C.c_size_t, C.c_uint64]),
    "poporon_bch_config_create": (_vp, [C.c_uint8, C.c_uint16, C.c_uint8]),
    "poporon_config_rs_default": (_vp, []),
    "poporon_config_ldpc_default": (_vp, [C.c_size_t, C.c_int]),
    "poporon_config_ldpc_burst_resistant": (_vp, [C.c_size_t, C.c_int]),
    "poporon_config_bch_default": (_vp, []),
    "poporon_config_destroy": (None, [_vp]),
    "poporon_create": (_vp, [_vp]),
    "poporon_destroy": (None, [_vp]),
    "poporon_encode": (C.c_bool, [_vp, _vp, C.c_size_t, _vp]),
    "poporon_decode": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.POINTER(C.c_size_t)]),
    "poporon_get_fec_type": (C.c_int, [_vp]),
    "poporon_get_iterations_used": (C.c_uint32, [_vp]),
    "poporon_get_parity_size": (C.c_size_t, [_vp]),
    "poporon_get_info_size": (C.c_size_t, [_vp]),
    "poporon_version_id": (C.c_uint32, []),
    "poporon_buildtime": (C.c_uint32, []),
    "poporon_erasure_create": (_vp, [C.c_uint16, C.c_uint32]),
    "poporon_erasure_create_from_positions": (_vp, [C.c_uint16, _vp, C.c_uint32]),
    "poporon_erasure_add_position": (C.c_bool, [_vp, C.c_uint32]),
    "poporon_erasure_reset": (None, [_vp]),
    "poporon_erasure_destroy": (None, [_vp]),
    "poporon_gf_create": (_vp, [C.c_uint8, C.c_uint16]),
    "poporon_gf_destroy": (None, [_vp]),
    "poporon_gf_mod": (C.c_uint8, [_vp, C.c_uint16]),
    "poporon_rs_create": (_vp, [C.c_uint8, C.c_uint16, C.c_uint16, C.c_uint16, C.c_uint8]),
    "poporon_rs_destroy": (None, [_vp]),
    "poporon_amd_last_error": (C.c_char_p, []),
    "poporon_amd_device_count": (C.c_int, []),
    "poporon_amd_set_device": (C.c_bool, [_vp, C.c_int]),
    "poporon_amd_reserve": (C.c_bool, [_vp, C.c_size_t]),
    "poporon_amd_supported": (C.c_bool, [_vp]),
    "poporon_amd_timing": (C.c_bool, [_vp, C.c_int]),
    "poporon_amd_timing_read": (C.c_bool, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "poporon_encode_batch_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t, _vp]),
    "poporon_decode_batch_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t, _vp,
                                               C.c_size_t, _vp, _vp, _vp, _vp]),
    "poporon_decode_batch_syndrome_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t,
                                                        C.c_size_t, _vp, C.c_size_t, _vp, _vp, _vp]),
    "poporon_check_batch_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t, _vp,
                                              _vp]),
    "poporon_encode_batch": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t]),
    "poporon_decode_batch": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t, _vp,
                                        C.c_size_t, _vp, _vp, _vp]),
    "poporon_rng_create": (_vp, [C.c_int, _vp, C.c_size_t]),
    "poporon_rng_destroy": (None, [_vp]),
    "poporon_rng_next": (C.c_bool, [_vp, _vp, C.c_size_t]),
    "poporon_amd_rng_fill_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp]),
    "poporon_syndrome_batch_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t,
                                                 _vp, C.c_size_t, _vp, _vp]),
    "poporon_amd_multi_create": (_vp, [_vp, _vp, C.c_size_t]),
    "poporon_amd_multi_destroy": (None, [_vp]),
    "poporon_amd_multi_device_count": (C.c_size_t, [_vp]),
    "poporon_amd_multi_handle": (_vp, [_vp, C.c_size_t]),
    "poporon_amd_multi_range": (C.c_bool, [C.c_size_t, C.c_size_t, C.c_size_t, C.POINTER(C.c_size_t),
                                           C.POINTER(C.c_size_t)]),
    "poporon_encode_batch_multi": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t]),
    "poporon_decode_batch_multi": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t, _vp,
                                              C.c_size_t, _vp, _vp, _vp]),
    "poporon_encode_batch_multi_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t,
                                                     _vp]),
    "poporon_decode_batch_multi_device": (C.c_bool, [_vp, _vp, C.c_size_t, _vp, C.c_size_t, C.c_size_t, C.c_size_t,
                                                     _vp, C.c_size_t, _vp, _vp, _vp, _vp]),
}

# kernel ids for poporon_amd_timing_read (include/poporon_amd.h)
KERNEL_ENCODE, KERNEL_REMAINDER, KERNEL_CORRECT = 0, 1, 2
KERNEL_BM, KERNEL_CHIEN, KERNEL_FORNEY, KERNEL_LIST, KERNEL_APPLY, KERNEL_ERASURE, KERNEL_SINGLE = 4, 5, 6, 7, 8, 9, 10
KERNEL_WAVE = 11
KERNEL_NAMES = {KERNEL_ENCODE: "rs_lfsr_k<false> (encode)", KERNEL_REMAINDER: "rs_lfsr_k<true> (remainder)",
                KERNEL_CORRECT: "rs_correct_k (BM/Chien/Forney)", KERNEL_BM: "rs_bm_k (BM/Omega)",
                KERNEL_CHIEN: "rs_chien_k (Chien)", KERNEL_FORNEY: "rs_forney_k (Forney)",
                KERNEL_APPLY: "rs_apply_k (apply)", KERNEL_LIST: "rs_wave_k (list)",
                KERNEL_ERASURE: "rs_era_bp_k (erasure)", KERNEL_SINGLE: "rs_dec1_k (one codeword)",
                KERNEL_WAVE: "rs_wave_k (small batch)"}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load the C-ABI library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not found: build it with `make -C libpoporon_amd` (hipcc, gfx950)")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If
    # this library bound /opt/rocm's copy first, torch's HIP init would fail,
    # so let torch (when installed) load the runtime and share it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def header_symbols(include_dir: str = INCLUDE_DIR):
    """Every function name declared in include/*.h and include/poporon/*.h."""
    names = []
    for sub in ("", "poporon"):
        d = os.path.join(include_dir, sub)
        for f in sorted(os.listdir(d)):
            if not f.endswith(".h"):
                continue
            text = open(os.path.join(d, f)).read()
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            for m in re.finditer(r"\b(poporon_[a-z0-9_]+)\s*\(", text):
                if m.group(1) not in names:
                    names.append(m.group(1))
    return names


def last_error() -> str:
    return load_library().poporon_amd_last_error().decode()


def device_count() -> int:
    return int(load_library().poporon_amd_device_count())


class PoporonError(RuntimeError):
    pass


def _buf(a):
    return a.ctypes.data_as(C.c_void_p)


def _u8(a, copy=False):
    if isinstance(a, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(a), dtype=np.uint8)
    return np.array(a, dtype=np.uint8, copy=True) if copy else np.ascontiguousarray(a, dtype=np.uint8)


class Erasure:
    """poporon_erasure_t (include/poporon/erasure.h), reference src/erasure.c."""

    def __init__(self, num_roots: int = 32, initial_capacity: int = 0, positions=None):
        self.lib = load_library()
        if positions is not None:
            arr = np.ascontiguousarray(positions, dtype=np.uint32)
            self.h = self.lib.poporon_erasure_create_from_positions(num_roots, _buf(arr), arr.size)
        else:
            self.h = self.lib.poporon_erasure_create(num_roots, initial_capacity)
        if not self.h:
            raise PoporonError("poporon_erasure_create returned NULL")

    def add(self, position: int) -> bool:
        return bool(self.lib.poporon_erasure_add_position(self.h, int(position)))

    def reset(self):
        self.lib.poporon_erasure_reset(self.h)

    def set(self, positions):
        self.reset()
        for p in positions:
            self.add(p)

    def close(self):
        if getattr(self, "h", None):
            self.lib.poporon_erasure_destroy(self.h)
            self.h = None

    __del__ = close


class Poporon:
    """A poporon_t RS handle (poporon_rs_config_create + poporon_create).

    ``erasure`` (an :class:`Erasure`) and ``syndrome`` (32 log-form values) are
    borrowed and read live at every single-codeword decode, as in the reference.
    """

    def __init__(self, symbol_size=8, generator_polynomial=0x11D, first_consecutive_root=1, primitive_element=1,
                 num_roots=32, erasure: Erasure | None = None, syndrome=None, device: int | None = None):
        self.lib = load_library()
        self.erasure = erasure
        self._syn = None
        if syndrome is not None:
            self._syn = np.ascontiguousarray(syndrome, dtype=np.uint16)
        cfg = self.lib.poporon_rs_config_create(symbol_size, generator_polynomial, first_consecutive_root,
                                                primitive_element, num_roots, erasure.h if erasure else None,
                                                _buf(self._syn) if self._syn is not None else None)
        if not cfg:
            raise PoporonError("poporon_rs_config_create returned NULL")
        self.h = self.lib.poporon_create(cfg)
        self.lib.poporon_config_destroy(cfg)
        if not self.h:
            raise PoporonError(f"poporon_create returned NULL {last_error()}")
        self.num_roots = num_roots
        if device is not None:
            self._check(self.lib.poporon_amd_set_device(self.h, device), "poporon_amd_set_device")

    @classmethod
    def default(cls, **kw):
        """poporon_config_rs_default(): RS(255,223), 0x11D, fcr 1, prim 1."""
        return cls(8, 0x11D, 1, 1, 32, **kw)

    def close(self):
        if getattr(self, "h", None):
            self.lib.poporon_destroy(self.h)
            self.h = None

    __del__ = close

    def _check(self, ok, what):
        if not ok:
            raise PoporonError(f"{what} failed: {last_error()}")

    # ---- getters ---------------------------------------------------------------
    @property
    def fec_type(self):
        return self.lib.poporon_get_fec_type(self.h)

    @property
    def parity_size(self):
        return self.lib.poporon_get_parity_size(self.h)

    @property
    def info_size(self):
        return self.lib.poporon_get_info_size(self.h)

    @property
    def supported(self):
        return bool(self.lib.poporon_amd_supported(self.h))

    # ---- single codeword (the reference's entry points) -------------------------
    def encode(self, data):
        """poporon_encode: returns the parity bytes (raises on failure)."""
        d = _u8(data)
        par = np.zeros(self.num_roots, np.uint8)
        self._check(self.lib.poporon_encode(self.h, _buf(d) if d.size else _buf(np.zeros(1, np.uint8)), d.size,
                                            _buf(par)), "poporon_encode")
        return par

    def decode(self, data, parity):
        """poporon_decode on copies: returns (ok, corrected_num, data', parity').

        A False result is a decode outcome (as in the reference), not an error,
        unless corrected_num == DEVICE_ERROR (a GPU failure; last_error() says which)."""
        d = _u8(data, copy=True)
        p = _u8(parity, copy=True)
        n = C.c_size_t(0)
        ok = self.lib.poporon_decode(self.h, _buf(d) if d.size else _buf(np.zeros(1, np.uint8)), d.size, _buf(p),
                                     C.byref(n))
        return bool(ok), int(n.value), d, p

    # ---- host batches ------------------------------------------------------------
    def encode_batch(self, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        count, size = data.shape
        par = np.zeros((count, self.num_roots), np.uint8)
        self._check(self.lib.poporon_encode_batch(self.h, _buf(data), size, _buf(par), self.num_roots, size, count),
                    "poporon_encode_batch")
        return par

    def decode_batch(self, data, parity, positions=None, counts=None):
        """Returns (ok u8[count], corrected u8[count], data', parity')."""
        d = np.array(data, dtype=np.uint8, copy=True, order="C")
        p = np.array(parity, dtype=np.uint8, copy=True, order="C")
        count, size = d.shape
        ok = np.zeros(count, np.uint8)
        cor = np.zeros(count, np.uint8)
        if positions is not None:
            pos = np.ascontiguousarray(positions, dtype=np.uint8)
            cnt = np.ascontiguousarray(counts, dtype=np.uint8)
            pargs = (_buf(pos), pos.shape[1], _buf(cnt))
        else:
            pargs = (None, 0, None)
        self._check(self.lib.poporon_decode_batch(self.h, _buf(d), size, _buf(p), p.shape[1], size, count, *pargs,
                                                  _buf(ok), _buf(cor)), "poporon_decode_batch")
        return ok, cor, d, p

    # ---- device batches (pointers + hipStream_t) ----------------------------------
    def encode_batch_device(self, d_data, data_stride, d_parity, parity_stride, size, count, stream=0):
        self._check(self.lib.poporon_encode_batch_device(self.h, d_data, data_stride, d_parity, parity_stride, size,
                                                         count, stream or None), "poporon_encode_batch_device")

    def decode_batch_device(self, d_data, data_stride, d_parity, parity_stride, size, count, d_ok, d_corrected=None,
                            d_positions=None, positions_stride=0, d_counts=None, stream=0):
        self._check(self.lib.poporon_decode_batch_device(self.h, d_data, data_stride, d_parity, parity_stride, size,
                                                         count, d_positions, positions_stride, d_counts, d_ok,
                                                         d_corrected, stream or None), "poporon_decode_batch_device")

    def decode_batch_syndrome_device(self, d_data, data_stride, d_parity, parity_stride, size, count, d_syndromes,
                                     syndrome_stride, d_ok, d_corrected=None, stream=0):
        """External-syndrome branch (src/decode.c:446-464) for a batch: d_syndromes holds num_roots
        u16 log-form syndromes per codeword, syndrome_stride elements apart."""
        self._check(self.lib.poporon_decode_batch_syndrome_device(self.h, d_data, data_stride, d_parity,
                                                                  parity_stride, size, count, d_syndromes,
                                                                  syndrome_stride, d_ok, d_corrected, stream or None),
                    "poporon_decode_batch_syndrome_device")

    def syndrome_batch_device(self, d_data, data_stride, d_parity, parity_stride, size, count, d_syndromes,
                              syndrome_stride, d_nonzero=None, stream=0):
        """calculate_syndrome_u8 for a batch: u16 log-form syndromes (+ nonzero flags)."""
        self._check(self.lib.poporon_syndrome_batch_device(self.h, d_data, data_stride, d_parity, parity_stride, size,
                                                           count, d_syndromes, syndrome_stride, d_nonzero,
                                                           stream or None), "poporon_syndrome_batch_device")

    def check_batch_device(self, d_data, data_stride, d_parity, parity_stride, size, count, d_dirty, stream=0):
        self._check(self.lib.poporon_check_batch_device(self.h, d_data, data_stride, d_parity, parity_stride, size,
                                                        count, d_dirty, stream or None), "poporon_check_batch_device")

    def reserve(self, max_count):
        self._check(self.lib.poporon_amd_reserve(self.h, max_count), "poporon_amd_reserve")

    # ---- in-library kernel timing (HIP events on the launch stream) ---------------
    def timing(self, enable: bool):
        self._check(self.lib.poporon_amd_timing(self.h, int(enable)), "poporon_amd_timing")

    def timing_read(self, kernel: int):
        ms = C.c_double(0)
        n = C.c_uint64(0)
        self._check(self.lib.poporon_amd_timing_read(self.h, kernel, C.byref(ms), C.byref(n)), "poporon_amd_timing_read")
        return ms.value, n.value


class Bch(Poporon):
    """A PPLN_FEC_BCH handle (poporon_bch_config_create + poporon_create): binary
    BCH over GF(2^m), messages and parity as big-endian byte images
    (src/encode.c:199-233, src/decode.c:542-590).  Same methods as
    :class:`Poporon`; ``parity_size``/``info_size`` are the byte-image sizes."""

    def __init__(self, symbol_size=4, generator_polynomial=0x13, correction_capability=3, device=None):
        self.lib = load_library()
        self.erasure = None
        self._syn = None
        cfg = self.lib.poporon_bch_config_create(symbol_size, generator_polynomial, correction_capability)
        if not cfg:
            raise PoporonError("poporon_bch_config_create returned NULL")
        self.h = self.lib.poporon_create(cfg)
        self.lib.poporon_config_destroy(cfg)
        if not self.h:
            raise PoporonError(f"poporon_create returned NULL {last_error()}")
        self.num_roots = int(self.lib.poporon_get_parity_size(self.h))  # parity bytes (array shapes)
        if device is not None:
            self._check(self.lib.poporon_amd_set_device(self.h, device), "poporon_amd_set_device")

    @classmethod
    def default(cls, **kw):
        """poporon_config_bch_default(): BCH(15, 5) over GF(16), 0x13, t = 3."""
        return cls(4, 0x13, 3, **kw)

    def decode(self, data, parity, corrected_init=0):
        """poporon_decode on copies: (ok, corrected_num, data').  As in the
        reference, corrected_num is left at corrected_init on failure."""
        d = _u8(data, copy=True)
        p = _u8(parity, copy=True)
        n = C.c_size_t(corrected_init)
        ok = self.lib.poporon_decode(self.h, _buf(d) if d.size else _buf(np.zeros(1, np.uint8)), d.size,
                                     _buf(p) if p.size else _buf(np.zeros(1, np.uint8)), C.byref(n))
        return bool(ok), int(n.value), d


class Rng:
    """poporon_rng_t (include/poporon/rng.h): xoshiro128++ seeded by splitmix32,
    reference src/rng.c.  ``next`` fills host memory; ``fill_device`` writes
    the same stream into device memory (poporon_amd_rng_fill_device)."""

    def __init__(self, seed: int | bytes | None = 0, rng_type: int = 0):
        self.lib = load_library()
        if seed is None:
            self.h = self.lib.poporon_rng_create(rng_type, None, 0)
        else:
            b = seed if isinstance(seed, (bytes, bytearray)) else int(seed).to_bytes(4, "little")
            buf = np.frombuffer(bytes(b), dtype=np.uint8).copy()
            self.h = self.lib.poporon_rng_create(rng_type, _buf(buf), buf.size)
        if not self.h:
            raise PoporonError("poporon_rng_create returned NULL")

    def next(self, size: int) -> np.ndarray:
        out = np.zeros(max(size, 1), np.uint8)
        if not self.lib.poporon_rng_next(self.h, _buf(out), size):
            raise PoporonError("poporon_rng_next failed")
        return out[:size]

    def fill_device(self, d_dest, size, stream=0):
        if not self.lib.poporon_amd_rng_fill_device(self.h, d_dest, size, stream or None):
            raise PoporonError(f"poporon_amd_rng_fill_device failed: {last_error()}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.poporon_rng_destroy(self.h)
            self.h = None

    __del__ = close


def shard_range(count: int, rank: int, world: int):
    """Contiguous codeword range [lo, hi) of `rank` out of `world`:
    the library's own partition (poporon_amd_multi_range), [count*r/W, count*(r+1)/W)."""
    first, n = C.c_size_t(0), C.c_size_t(0)
    if not load_library().poporon_amd_multi_range(count, world, rank, C.byref(first), C.byref(n)):
        raise PoporonError(f"poporon_amd_multi_range failed: {last_error()}")
    return int(first.value), int(first.value + n.value)


class Multi:
    """poporon_multi_t (include/poporon_amd.h): one RS handle per device, each
    codeword range on its own device; host batches run the devices concurrently."""

    def __init__(self, devices=None, symbol_size=8, generator_polynomial=0x11D, first_consecutive_root=1,
                 primitive_element=1, num_roots=32):
        self.lib = load_library()
        cfg = self.lib.poporon_rs_config_create(symbol_size, generator_polynomial, first_consecutive_root,
                                                primitive_element, num_roots, None, None)
        if not cfg:
            raise PoporonError("poporon_rs_config_create returned NULL")
        if devices is None:
            self.h = self.lib.poporon_amd_multi_create(cfg, None, 0)
        else:
            arr = (C.c_int * len(devices))(*devices)
            self.h = self.lib.poporon_amd_multi_create(cfg, arr, len(devices))
        self.lib.poporon_config_destroy(cfg)
        if not self.h:
            raise PoporonError(f"poporon_amd_multi_create failed: {last_error()}")
        self.num_roots = num_roots

    @property
    def devices(self):
        return int(self.lib.poporon_amd_multi_device_count(self.h))

    def _check(self, ok, what):
        if not ok:
            raise PoporonError(f"{what} failed: {last_error()}")

    def encode_batch(self, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        count, size = data.shape
        par = np.zeros((count, self.num_roots), np.uint8)
        self._check(self.lib.poporon_encode_batch_multi(self.h, _buf(data), size, _buf(par), self.num_roots, size,
                                                        count), "poporon_encode_batch_multi")
        return par

    def decode_batch(self, data, parity, positions=None, counts=None):
        d = np.array(data, dtype=np.uint8, copy=True, order="C")
        p = np.array(parity, dtype=np.uint8, copy=True, order="C")
        count, size = d.shape
        ok = np.zeros(count, np.uint8)
        cor = np.zeros(count, np.uint8)
        if positions is not None:
            pos = np.ascontiguousarray(positions, dtype=np.uint8)
            cnt = np.ascontiguousarray(counts, dtype=np.uint8)
            pargs = (_buf(pos), pos.shape[1], _buf(cnt))
        else:
            pargs = (None, 0, None)
        self._check(self.lib.poporon_decode_batch_multi(self.h, _buf(d), size, _buf(p), p.shape[1], size, count,
                                                        *pargs, _buf(ok), _buf(cor)), "poporon_decode_batch_multi")
        return ok, cor, d, p

    def encode_batch_device(self, d_data, data_stride, d_parity, parity_stride, size, count, streams=None):
        """d_data / d_parity / streams: one pointer per device (device i's range of rows)."""
        G = self.devices
        arr = lambda v: (C.c_void_p * G)(*v)  # noqa: E731
        self._check(self.lib.poporon_encode_batch_multi_device(self.h, arr(d_data), data_stride, arr(d_parity),
                                                               parity_stride, size, count,
                                                               arr(streams) if streams else None),
                    "poporon_encode_batch_multi_device")

    def decode_batch_device(self, d_data, data_stride, d_parity, parity_stride, size, count, d_ok, d_corrected=None,
                            streams=None, d_positions=None, positions_stride=0, d_counts=None):
        """d_positions / d_counts (erasure batches): one pointer per device, as d_data."""
        G = self.devices
        arr = lambda v: (C.c_void_p * G)(*v)  # noqa: E731
        self._check(self.lib.poporon_decode_batch_multi_device(self.h, arr(d_data), data_stride, arr(d_parity),
                                                               parity_stride, size, count,
                                                               arr(d_positions) if d_positions else None,
                                                               positions_stride,
                                                               arr(d_counts) if d_counts else None, arr(d_ok),
                                                               arr(d_corrected) if d_corrected else None,
                                                               arr(streams) if streams else None),
                    "poporon_decode_batch_multi_device")

    def close(self):
        if getattr(self, "h", None):
            self.lib.poporon_amd_multi_destroy(self.h)
            self.h = None

    __del__ = close
