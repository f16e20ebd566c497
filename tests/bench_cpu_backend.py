"""CPU stand-in for bench.py's GPU backend (TEST INFRASTRUCTURE ONLY).

The gloo launcher test (tests/test_distributed_cpu.py) runs
`bench.py --gpus 2 --backend tests.bench_cpu_backend`: the same launcher,
partition, configs[4] strong split and rank reductions as the GPU run, with
the codec replaced by the CPU oracle (oracle/rs_oracle.c, pinned to the
reference's fixtures) and the synthesis / channel / checksum by testutil's
numpy restatements of its HIP kernels.
"""
import numpy as np

import testutil as T
from oracle import Oracle

K, NR, N = 223, 32, 255
SEED = 0x5EED0001


class Backend:
    kind = "cpu"
    dist_backend = "gloo"

    def __init__(self, local):
        self.o = Oracle()

    def sync(self):
        pass

    def rows(self, n):
        return np.zeros((n, N), np.uint8)

    def like(self, buf):
        return np.empty_like(buf)

    def copy(self, dst, src):
        dst[...] = src

    def synth_messages(self, buf, first, seed=SEED):
        buf[:, :K] = T.synth_rows_cpu(seed, first, buf.shape[0], K)

    def errors(self, first, n, nerr, span, seed, sorted_positions=False):
        return T.synth_errors_cpu(seed, first, n, nerr, span, sorted_positions)

    def channel(self, buf, err):
        pos, mag = err
        buf[...] = T.channel_xor_cpu(buf, pos, mag)

    def encode(self, buf, side=False):
        buf[:, K:] = self.o.encode_batch(np.ascontiguousarray(buf[:, :K]))

    def status(self, n):
        return np.zeros(n, np.uint8), np.zeros(n, np.uint8)

    def decode(self, buf, st, erasures=None):
        assert erasures is None
        ok, cor, d, p = self.o.decode_batch(np.ascontiguousarray(buf[:, :K]), np.ascontiguousarray(buf[:, K:]))
        buf[:, :K], buf[:, K:] = d, p
        st[0][:], st[1][:] = ok, cor

    def counts(self, n, v):
        return np.full(n, v, np.uint8)

    def checksum(self, buf, first):
        return T.checksum_cpu(buf, first)

    def n_bad(self, st, want_cor):
        ok, cor = st
        return int((ok != 1).sum()) + int((cor != want_cor).sum())

    def n_diff(self, a, b):
        return int((a != b).any(axis=1).sum())

    def host(self, t, idx):
        return np.asarray(t)[idx].copy()

    def from_host(self, a):
        return a.copy()

    def mask_errors(self, mag, ne):
        mag[np.arange(mag.shape[1])[None, :] >= ne[:, None]] = 0

    def n_bad_mixed(self, st, ne, out, clean):
        ok, cor = st
        return int(((ne <= 16) & ((ok != 1) | (cor != ne) | (out != clean).any(1))).sum())

    def count_ok(self, st):
        return int(st[0].sum())

    def free_bytes(self):
        return 1 << 40
