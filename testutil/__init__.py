"""testutil -- test and benchmark utilities for libpoporon_amd (not the codec).

``libpoporon_testutil.so`` (``testutil.hip``) generates synthetic payloads and
error patterns on the device, applies the symbol-error channel and checksums
row batches.  Every value depends only on (seed, global row index), so a batch
sharded over ranks reproduces the single-process batch row for row.  The
numpy functions here restate each formula for CPU-side tests (and for the gloo
launcher test of bench.py); ``tests/test_gpu_parity.py`` checks both agree.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpoporon_testutil.so")

_K32 = 0x9E3779B1
_M32 = 0xFFFFFFFF
_M64 = (1 << 64) - 1
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `make -C testutil`")
        try:
            import torch  # noqa: F401  (one HIP runtime per process: torch's)
        except ImportError:
            pass
        lib = C.CDLL(LIB_PATH)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        sigs = {
            "ptu_synth_rows": [u32, u64, u64, u32, vp, u64, vp],
            "ptu_synth_errors": [u32, u64, u64, u32, u32, C.c_int, vp, vp, vp],
            "ptu_channel_xor": [vp, vp, u64, vp, u64, u64, vp],
            "ptu_checksum": [vp, u64, u32, u64, u64, vp, vp],
        }
        for name, args in sigs.items():
            fn = getattr(lib, name)
            fn.restype = C.c_bool
            fn.argtypes = args
        lib.ptu_time_encode.restype = lib.ptu_time_decode.restype = C.c_double
        lib.ptu_time_encode.argtypes = [vp, vp, vp, u64, vp, u64, u64]
        lib.ptu_time_decode.argtypes = [vp, vp, vp, u64, vp, u64, u64, u64, vp, vp]
        _lib = lib
    return _lib


def _ok(r, what):
    if not r:
        raise RuntimeError(f"{what} failed")


# ---- device (HIP) ----------------------------------------------------------
def synth_rows(seed, first, count, width, d_out, stride, stream=0):
    _ok(load().ptu_synth_rows(seed, first, count, width, d_out, stride, stream or None), "ptu_synth_rows")


def synth_errors(seed, first, count, nerr, span, d_pos, d_mag, sorted_positions=False, stream=0):
    _ok(load().ptu_synth_errors(seed, first, count, nerr, span, int(sorted_positions), d_pos, d_mag, stream or None),
        "ptu_synth_errors")


def channel_xor(d_pos, d_mag, per_row, d_rows, stride, count, stream=0):
    _ok(load().ptu_channel_xor(d_pos, d_mag, per_row, d_rows, stride, count, stream or None), "ptu_channel_xor")


def _vp(a):
    return a.ctypes.data_as(C.c_void_p)


def time_encode(lib, h, msgs, par):
    """A C loop of lib.poporon_encode (lib: a ctypes CDLL) on handle h:
    msgs[c] (size bytes) -> par[c]; returns seconds (< 0: a call failed)."""
    n, size = msgs.shape
    return load().ptu_time_encode(C.cast(lib.poporon_encode, C.c_void_p), h, _vp(msgs), size, _vp(par), par.shape[1],
                                  n)


def time_decode(lib, h, data, par):
    """A C loop of lib.poporon_decode on handle h over the rows data[c] /
    par[c], decoded in place; returns (seconds, ok u8[n], corrected u8[n])."""
    n, size = data.shape
    ok = np.zeros(n, np.uint8)
    cor = np.zeros(n, np.uint8)
    t = load().ptu_time_decode(C.cast(lib.poporon_decode, C.c_void_p), h, _vp(data), size, _vp(par), par.shape[1],
                               size, n, _vp(ok), _vp(cor))
    return t, ok, cor


def checksum(d_rows, stride, width, first, count, d_sum, stream=0):
    """*d_sum += checksum (d_sum: device uint64, caller-initialised)."""
    _ok(load().ptu_checksum(d_rows, stride, width, first, count, d_sum, stream or None), "ptu_checksum")


# ---- the same formulas in numpy (CPU) ---------------------------------------
def _fmix32(x):
    x = x.astype(np.uint64) & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(_M32)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(_M32)
    return x ^ (x >> np.uint64(16))


def _fmix64(x):
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xFF51AFD7ED558CCD)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xC4CEB9FE1A85EC53)
        return x ^ (x >> np.uint64(33))


def synth_rows_cpu(seed, first, count, width):
    """uint8[count, width]: byte j of row i = fmix32(((first+i)*width + j) * K + seed) & 255."""
    rows = np.arange(first, first + count, dtype=np.uint64)[:, None]
    ctr = (rows * np.uint64(width) + np.arange(width, dtype=np.uint64)[None, :]) & np.uint64(_M32)
    return (_fmix32((ctr * np.uint64(_K32) + np.uint64(seed)) & np.uint64(_M32)) & np.uint64(255)).astype(np.uint8)


def synth_errors_cpu(seed, first, count, nerr, span, sorted_positions=False):
    """(pos uint8[count, nerr], mag uint8[count, nerr]) as ptu_synth_errors."""
    rows = np.arange(first, first + count, dtype=np.uint64)[:, None]
    ctr = (rows * np.uint64(span) + np.arange(span, dtype=np.uint64)[None, :]) & np.uint64(_M32)
    keys = _fmix32((ctr * np.uint64(_K32) + np.uint64(seed)) & np.uint64(_M32))
    pos = np.argsort(-keys.astype(np.int64), axis=1, kind="stable")[:, :nerr]
    mctr = (rows * np.uint64(nerr) + np.arange(nerr, dtype=np.uint64)[None, :]) & np.uint64(_M32)
    mag = (_fmix32((mctr * np.uint64(_K32) + np.uint64(seed + 0x1234567)) & np.uint64(_M32)) % np.uint64(255) +
           np.uint64(1))
    if sorted_positions:
        order = np.argsort(pos, axis=1, kind="stable")
        pos = np.take_along_axis(pos, order, 1)
        mag = np.take_along_axis(mag, order, 1)
    return pos.astype(np.uint8), mag.astype(np.uint8)


def channel_xor_cpu(rows, pos, mag):
    out = rows.copy()
    r = np.arange(rows.shape[0])[:, None]
    out[r, pos.astype(np.int64)] ^= mag
    return out


def checksum_cpu(rows, first):
    """uint64 checksum of uint8[count, width] rows starting at global row `first` (as ptu_checksum)."""
    count, width = rows.shape
    with np.errstate(over="ignore"):
        idx = np.arange(first, first + count, dtype=np.uint64)
        h = _fmix64(idx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(width))
        for j in range(width):
            h = (h ^ rows[:, j].astype(np.uint64)) * np.uint64(0x100000001B3)
        h = _fmix64(h)
        return int(h.sum(dtype=np.uint64))
