#!/usr/bin/env python3
"""bench.py -- RS(255,223) encode + decode@16 throughput on MI355X.

One step = one pass of the hot path over one batch of synthetic codewords
resident in HBM (configs[1] + configs[2] of BASELINE.json, chained):

    encode  2^20 messages x 223 B -> 32 parity bytes each        (HIP, C ABI)
    decode  2^20 codewords with 16 errors each (unique positions over all 255
            bytes, magnitudes in [1,255]): syndromes/BM/Chien/Forney/apply,
            in place                                             (HIP, C ABI)

The errors come from the test channel (testutil/, not part of the codec):
before the timed loop it corrupts one copy of the encoded batch per step, and
step k decodes copy k, so every step does the full decode work and the timed
loop holds only codec kernels.  Codeword layout: one 255-byte row per codeword
(data then parity), stride 255.  value = codewords through encode + decode per
second, summed over all ranks (weak scaling: --batch codewords per GPU).
Inputs are generated on the device from a counter hash of (seed, global
codeword index), so any sharding sees the same codewords.

configs[4] (strong split): --c4-total codewords (default 2^26) are split into
contiguous ranges over the ranks (libpoporon_amd's own partition); each rank
encodes, corrupts (untimed) and decodes its range; the line reports their
cw/s (max-over-ranks time) and a checksum of every decoded codeword that is
identical for every GPU count.  --c4-scatter T (opt-in, N > 1) adds the split
as a data movement: rank 0 holds T corrupted codewords and sends each rank its
range point-to-point (RCCL send/recv over xGMI) before every rank decodes it.

Multi-GPU: `bench.py --gpus N` starts N ranks itself (torch.distributed.run as
a child process, before anything touches the GPU) unless it already runs
under a launcher (WORLD_SIZE set, which must equal N).  One process per GPU,
RCCL (`nccl` backend) only for barriers and the max-time / checksum
reductions; no data-path collective (but for the opt-in --c4-scatter).

Also reported: per-kernel HIP-event times (in-library, stamped by each kernel's dispatch),
the roofline of the dominant kernel, erasure decode (configs[3]), the
host-memory pipeline (PCIe-inclusive), single-codeword call latency, and the
reference CPU path timed on the host cores (rank 0, N=1 only).

--backend MODULE replaces the GPU codec by MODULE.Backend (tests only: the
gloo launcher test runs the same launcher, partition and reduction code on
CPU with tests/bench_cpu_backend.py).

POPORON_BENCH_ONE_DEVICE=1 (rehearsal only, never a scaling number): every
rank on cuda:0 with gloo reductions on host tensors, so the N > 1 GPU path
(launcher, per-rank ranges, kernels, per-rank reports, checksums) runs on a
one-GPU box; the line says so under "rehearsal".
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "RS(255,223) codewords/s (encode; decode @ t=16 errs) and GB/s vs HBM peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CW_BYTES = 255         # algorithmic bytes per codeword
K, NR, N = 223, 32, 255
SEED = 0x5EED0001      # messages; errors: SEED + 1; erasures: SEED + 2; configs[4]: SEED + 4 / + 5; mixed: + 9 / + 10
MIXED_P, MIXED_CAP = 0.045, 24  # the mixed channel: binomial(255, p) errors per codeword, capped
M64 = (1 << 64) - 1


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--overlap", type=int, default=0,
                    help="1: each step's encode on a second stream, concurrent with its decode")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per GPU (weak-scaling line)")
    ap.add_argument("--c4-total", type=int, default=1 << 26, help="configs[4]: codewords split over all ranks")
    ap.add_argument("--c4-chunk", type=int, default=1 << 24, help="configs[4]: codewords per rank-chunk (memory)")
    ap.add_argument("--c4-reps", type=int, default=2)
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--c4-scatter", type=int, default=0,
                    help="configs[4] as a data movement (N > 1, opt-in): rank 0 holds this many corrupted codewords "
                         "and sends each rank its range point-to-point (RCCL send/recv over xGMI), then every rank "
                         "decodes its range")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-erasure", action="store_true")
    ap.add_argument("--no-mixed", action="store_true", help="skip the mixed-channel decode (binomial error counts)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory (PCIe) pipeline rates")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-codeword call latency")
    ap.add_argument("--no-general", action="store_true", help="skip the general-parameter RS(255,239) line")
    ap.add_argument("--backend", default="", help="tests only: module with a CPU Backend (see docstring)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="HBM bytes per codeword of each path from rocprofv3 --pmc passes (tools/pmc_traffic.py), "
                         "used only when stamped with the current kernel sources")
    ap.add_argument("--enc-copies", type=int, default=3,
                    help="message buffers the timed encode rotates over (3 x 267 MB >= 2 x the 256 MB MALL)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------
# paths (255 algorithmic bytes per codeword per mode)
# ----------------------------------------------------------------------------
# kernel ids of include/poporon_amd.h (POPORON_AMD_KERNEL_*) that make up each
# mode's path; a path's time per step is the sum of its kernels' times
K_ENCODE, K_REMAINDER, K_CORRECT, K_CHECK, K_BM, K_CHIEN, K_FORNEY, K_LIST, K_APPLY, K_ERASURE, K_SINGLE = range(11)
PATHS = {
    "encode": (K_ENCODE,),
    "decode16": (K_REMAINDER, K_BM, K_CHIEN, K_FORNEY, K_APPLY, K_LIST, K_CORRECT),
    "erasure32": (K_REMAINDER, K_ERASURE, K_BM, K_CHIEN, K_FORNEY, K_LIST, K_APPLY, K_CORRECT),
    "errata16e8": (K_REMAINDER, K_ERASURE, K_BM, K_CHIEN, K_FORNEY, K_LIST, K_APPLY, K_CORRECT),
    "decode_mixed": (K_REMAINDER, K_BM, K_CHIEN, K_FORNEY, K_APPLY, K_LIST, K_CORRECT),
}


def source_stamp():
    """Hash of the product kernel sources: a PMC traffic file is used only by
    a bench of the same kernels (tools/pmc_traffic.py writes the stamp)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "libpoporon_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*"))):
        if f.endswith((".hip", ".h", ".cpp")):
            h.update(os.path.basename(f).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def load_traffic(path):
    """{mode: HBM bytes per codeword} from a traffic file stamped with the
    current sources; (None, reason) otherwise."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "no traffic file"
    if t.get("source_stamp") != source_stamp():
        return None, f"stale: traffic file stamp {t.get('source_stamp')} != kernel sources {source_stamp()}"
    return t, None


def path_roofline(mode, kt, steps, B, traffic):
    """Path-level roofline of one mode: 255 B x codewords per step / the sum of
    the mode's kernel times per step (HIP events stamped by the kernels' dispatches on the launch stream)."""
    ks = [k for k in PATHS[mode] if k in kt and kt[k][1]]
    ms = sum(kt[k][0] / steps for k in ks)
    if ms <= 0:
        return None
    achieved = B * CW_BYTES / (ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "path_ms": round(ms, 4),
         "kernels_ms": {k: round(kt[k][0] / steps, 4) for k in ks}, "codewords": B,
         "algorithmic_bytes": B * CW_BYTES}
    if traffic is not None:
        m = traffic.get("modes", {}).get(mode)
        if m and m.get("hbm_bytes_per_cw"):
            r["traffic"] = round(m["hbm_bytes_per_cw"] * B)
            r["traffic_ratio"] = round(m["hbm_bytes_per_cw"] / CW_BYTES, 3)
    return r


# ----------------------------------------------------------------------------
# launcher: N ranks from one command, before any GPU use
# ----------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) outside a launcher: run N ranks under
    torch.distributed.run as a CHILD process (this process has not touched
    the GPU and never execs) and return its exit code; None when this
    process is itself a rank."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def one_device():
    """rehearsal: every rank on cuda:0, gloo (module docstring)"""
    return os.environ.get("POPORON_BENCH_ONE_DEVICE") == "1"


def dist_setup(backend_name):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend_name == "nccl" and one_device():
        if world > 1:
            dist.init_process_group(backend="gloo")
        torch.cuda.set_device(0)
        return world, rank, 0
    if world > 1:
        if backend_name == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend="gloo")
    elif backend_name == "nccl":
        torch.cuda.set_device(0)
    return world, rank, local


class Ranks:
    """Barrier / reductions over the ranks (RCCL on GPU, gloo on CPU tests)."""

    def __init__(self, world, device):
        import torch
        import torch.distributed as dist
        self.world, self.device, self.torch, self.dist = world, device, torch, dist
        self.rank = dist.get_rank() if world > 1 else 0

    def scatter_rows(self, out, chunks):
        """Rank 0 sends chunks[r] to rank r point-to-point (RCCL send/recv:
        over xGMI between GPUs; gloo on CPU tests) and copies chunks[0]
        into its own `out`; every other rank receives into `out`."""
        torch, dist = self.torch, self.dist
        t = lambda a: a if isinstance(a, torch.Tensor) else torch.from_numpy(a)  # noqa: E731
        if self.rank == 0:
            ops = [dist.P2POp(dist.isend, t(chunks[r]), r) for r in range(1, self.world)]
            t(out).copy_(t(chunks[0]))
        else:
            ops = [dist.P2POp(dist.irecv, t(out), 0)]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()

    def barrier(self, sync):
        sync()
        if self.world > 1:
            self.dist.barrier()
        sync()

    def max(self, x):
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.device)
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_int(self, x):
        t = self.torch.tensor([int(x)], dtype=self.torch.int64, device=self.device)
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return int(t.item())

    def gather(self, xs, dtype):
        """every rank's list xs (same length on every rank), in rank order"""
        t = self.torch.tensor(list(xs), dtype=dtype, device=self.device)
        if self.world == 1:
            return [t.tolist()]
        out = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]

    def sum_u64(self, x):
        """sum mod 2^64 of unsigned 64-bit values (carried as two's-complement int64)"""
        v = int(x) & M64
        s = self.sum_int(v - (1 << 64) if v >= (1 << 63) else v)
        return s & M64


# ----------------------------------------------------------------------------
# GPU backend: libpoporon_amd (the product, C ABI) + testutil (synthesis,
# channel, checksum; not the codec)
# ----------------------------------------------------------------------------
class GpuBackend:
    kind = "gpu"
    dist_backend = "nccl"

    def __init__(self, local):
        import torch

        import libpoporon_amd as P
        import testutil as T
        self.torch, self.P, self.T = torch, P, T
        self.dev = torch.device("cuda", local)
        self.local = local
        self.rs = P.Poporon.default(device=local)
        self.stream = torch.cuda.current_stream().cuda_stream

    def sync(self):
        self.torch.cuda.synchronize()

    def rows(self, n):
        return self.torch.empty((n, N), dtype=self.torch.uint8, device=self.dev)

    def like(self, buf):
        return self.torch.empty_like(buf)

    def copy(self, dst, src):
        dst.copy_(src)

    def synth_messages(self, buf, first, seed=SEED):
        self.T.synth_rows(seed, first, buf.shape[0], K, buf.data_ptr(), N, self.stream)

    def errors(self, first, n, nerr, span, seed, sorted_positions=False):
        pos = self.torch.empty((n, nerr), dtype=self.torch.uint8, device=self.dev)
        mag = self.torch.empty((n, nerr), dtype=self.torch.uint8, device=self.dev)
        self.T.synth_errors(seed, first, n, nerr, span, pos.data_ptr(), mag.data_ptr(), sorted_positions, self.stream)
        return pos, mag

    def channel(self, buf, err):
        pos, mag = err
        self.T.channel_xor(pos.data_ptr(), mag.data_ptr(), pos.shape[1], buf.data_ptr(), N, buf.shape[0], self.stream)

    def encode(self, buf, side=False):
        """side=True: on a second stream (the caller orders it: the step's
        encode and decode touch different buffers and may run concurrently)"""
        b = buf.data_ptr()
        s = self.stream
        if side:
            if getattr(self, "side_stream", None) is None:
                self.side = self.torch.cuda.Stream(device=self.dev)
                self.side_stream = self.side.cuda_stream
            s = self.side_stream
        self.rs.encode_batch_device(b, N, b + K, N, K, buf.shape[0], s)

    def status(self, n):
        return (self.torch.zeros(n, dtype=self.torch.uint8, device=self.dev),
                self.torch.zeros(n, dtype=self.torch.uint8, device=self.dev))

    def decode(self, buf, st, erasures=None):
        b = buf.data_ptr()
        ok, cor = st
        if erasures is None:
            self.rs.decode_batch_device(b, N, b + K, N, K, buf.shape[0], ok.data_ptr(), cor.data_ptr(),
                                        stream=self.stream)
        else:
            slots, cnts = erasures
            self.rs.decode_batch_device(b, N, b + K, N, K, buf.shape[0], ok.data_ptr(), cor.data_ptr(),
                                        d_positions=slots.data_ptr(), positions_stride=slots.shape[1],
                                        d_counts=cnts.data_ptr(), stream=self.stream)

    def counts(self, n, v):
        return self.torch.full((n,), v, dtype=self.torch.uint8, device=self.dev)

    def checksum(self, buf, first):
        s = self.torch.zeros(1, dtype=self.torch.int64, device=self.dev)
        self.T.checksum(buf.data_ptr(), N, N, first, buf.shape[0], s.data_ptr(), self.stream)
        return int(s.item()) & M64

    def n_bad(self, st, want_cor):
        ok, cor = st
        return int((ok != 1).sum()) + int((cor != want_cor).sum())

    def n_diff(self, a, b):
        return int((a != b).any(dim=1).sum())

    def host(self, t, idx):
        """rows idx of a device tensor, as numpy"""
        return t[self.torch.as_tensor(idx, device=self.dev)].cpu().numpy()

    def from_host(self, a):
        return self.torch.from_numpy(a).to(self.dev)

    def mask_errors(self, mag, ne):
        """zero the magnitudes past each row's error count (the channel then skips them)"""
        k = self.torch.arange(mag.shape[1], device=self.dev)
        mag.mul_((k[None, :] < ne[:, None].long()).to(self.torch.uint8))

    def n_bad_mixed(self, st, ne, out, clean):
        """codewords with <= 16 errors not restored with ok = 1 and corrected = their count"""
        ok, cor = st
        bad = (ne <= 16) & ((ok != 1) | (cor != ne) | (out != clean).any(dim=1))
        return int(bad.sum())

    def count_ok(self, st):
        return int(st[0].sum())

    def free_bytes(self):
        return self.torch.cuda.mem_get_info(self.dev)[0]


# ----------------------------------------------------------------------------
# configs[4]: strong split of --c4-total codewords over the ranks
# ----------------------------------------------------------------------------
def shard(total, rank, world):
    """The library's partition (poporon_amd_multi_range): [total*r/W, total*(r+1)/W)."""
    return total * rank // world, total * (rank + 1) // world


def run_strong(be, ranks, args, rank, world):
    import numpy as np
    lo, hi = shard(args.c4_total, rank, world)
    t_codec, nbad, csum_in, csum_out = 0.0, 0, 0, 0
    chunk = max(1, args.c4_chunk)
    reps = max(1, args.c4_reps)
    # parity sample: every C4_SAMPLE_STRIDE-th global codeword of the first
    # repetition (its encode and its decode), checked after the timed loops
    senc, sdec = {"msg": [], "got_par": []}, {"in": [], "out": [], "ok": [], "cor": []}
    for rep in range(reps):
        t_rep = 0.0
        for a in range(lo, hi, chunk):
            n = min(chunk, hi - a)
            buf = be.rows(n)
            be.synth_messages(buf, a, seed=SEED + 4)
            be.sync()
            t0 = time.perf_counter()
            be.encode(buf)
            be.sync()
            t_rep += time.perf_counter() - t0
            idx = np.arange((-a) % C4_SAMPLE_STRIDE, n, C4_SAMPLE_STRIDE, dtype=np.int64)
            if rep == 0:
                csum_in = (csum_in + be.checksum(buf, a)) & M64
                rows = be.host(buf, idx)
                senc["msg"].append(rows[:, :K])
                senc["got_par"].append(rows[:, K:])
            err = be.errors(a, n, 16, N, SEED + 5)
            be.channel(buf, err)
            del err
            st = be.status(n)
            if rep == 0:
                sdec["in"].append(be.host(buf, idx))
            be.sync()
            t0 = time.perf_counter()
            be.decode(buf, st)
            be.sync()
            t_rep += time.perf_counter() - t0
            if rep == 0:
                nbad += be.n_bad(st, 16)
                csum_out = (csum_out + be.checksum(buf, a)) & M64
                sdec["out"].append(be.host(buf, idx))
                sdec["ok"].append(be.host(st[0], idx))
                sdec["cor"].append(be.host(st[1], idx))
            del buf, st
        t_codec = t_rep if rep == 0 else min(t_codec, t_rep)
    t = ranks.max(t_codec)
    cs_in, cs_out = ranks.sum_u64(csum_in), ranks.sum_u64(csum_out)
    nbad = ranks.sum_int(nbad)
    # each rank's share of the checksum (u64 as two's-complement int64): their
    # sum mod 2^64 is parity_checksum, the same for every N
    s64 = lambda v: v - (1 << 64) if v >= (1 << 63) else v  # noqa: E731
    rank_cs = [[c & M64 for c in r] for r in ranks.gather([s64(csum_in & M64), s64(csum_out & M64)], ranks.torch.int64)]
    return {"total_codewords": args.c4_total, "codewords_per_gpu": hi - lo, "n_gpus": world,
            "cw_per_s": round(args.c4_total / t, 1) if t > 0 else None,
            "GB_per_s": round(args.c4_total * CW_BYTES / t / 1e9, 2) if t > 0 else None,
            "ms": round(t * 1e3, 3), "split": "contiguous ranges [T*r/N, T*(r+1)/N)",
            "timed": f"encode + decode@16 of each rank's range (best of {reps}), max over ranks; "
                     "synthesis, channel and checksums untimed",
            "verified": nbad == 0 and cs_in == cs_out and sum(r[1] for r in rank_cs) & M64 == cs_out,
            "parity_checksum": cs_out,
            "rank_checksums": [{"rank": i, "range": list(shard(args.c4_total, i, world)), "in": r[0], "out": r[1]}
                               for i, r in enumerate(rank_cs)],
            "_samples": {"configs4_encode": {k: np.concatenate(v) for k, v in senc.items()},
                         "configs4_decode16": {k: np.concatenate(v) for k, v in sdec.items()}}}


def run_scatter(be, ranks, args, rank, world):
    """configs[4]'s "batch split" with the data movement in it (opt-in,
    --c4-scatter T): rank 0 holds T encoded and corrupted codewords (16
    errors each) and sends rank r its range [T*r/N, T*(r+1)/N) point-to-point
    (RCCL send/recv: the xGMI links from GPU 0), then every rank decodes its
    range.  Timed: scatter, and scatter + decode, max over ranks (best of
    --c4-reps; the first exchange sets up the P2P channels).  Verified: every
    codeword decoded with ok = 1, corrected = 16, and the checksum of all
    decoded codewords equal to that of the encoded batch."""
    total = args.c4_scatter
    lo, hi = shard(total, rank, world)
    mine = be.rows(hi - lo)
    chunks, csum_clean = None, 0
    if rank == 0:
        src = be.rows(total)
        be.synth_messages(src, 0, seed=SEED + 11)
        be.encode(src)
        csum_clean = be.checksum(src, 0)
        err = be.errors(0, total, 16, N, SEED + 12)
        be.channel(src, err)
        del err
        chunks = [src[shard(total, r, world)[0]:shard(total, r, world)[1]] for r in range(world)]
    st = be.status(hi - lo)
    t_sc, t_all = None, None
    for _ in range(max(2, args.c4_reps)):
        ranks.barrier(be.sync)
        t0 = time.perf_counter()
        ranks.scatter_rows(mine, chunks)
        be.sync()
        t1 = time.perf_counter()
        be.decode(mine, st)
        be.sync()
        t2 = time.perf_counter()
        a, b = ranks.max(t1 - t0), ranks.max(t2 - t0)
        t_sc, t_all = (a, b) if t_sc is None else (min(t_sc, a), min(t_all, b))
    nbad = ranks.sum_int(be.n_bad(st, 16))
    cs_out = ranks.sum_u64(be.checksum(mine, lo))
    cs_in = ranks.sum_u64(csum_clean)
    moved = (total - shard(total, 0, world)[1]) * N  # bytes that leave rank 0
    return {"total_codewords": total, "n_gpus": world, "split": "contiguous ranges [T*r/N, T*(r+1)/N) from rank 0",
            "scatter_ms": round(t_sc * 1e3, 3), "scatter_GB_per_s": round(moved / t_sc / 1e9, 2) if t_sc > 0 else None,
            "scatter_decode_ms": round(t_all * 1e3, 3),
            "cw_per_s": round(total / t_all, 1) if t_all > 0 else None,
            "timed": "send/recv of the ranges + decode@16 of each range, max over ranks; synthesis, encode and "
                     "channel on rank 0 untimed",
            "verified": nbad == 0 and cs_in == cs_out, "parity_checksum": cs_out}


# ----------------------------------------------------------------------------
# weak-scaling line: --batch codewords per rank, encode + decode per step
# ----------------------------------------------------------------------------
def run_weak(be, ranks, args, rank, world):
    B = args.batch
    first = rank * B
    cw = be.rows(B)
    be.synth_messages(cw, first)
    err = be.errors(first, B, 16, N, SEED + 1)
    st = be.status(B)
    be.encode(cw)
    be.sync()
    clean = be.like(cw)
    be.copy(clean, cw)
    ncopy = args.warmup + 2 * args.steps  # two timed loops (plain, then with kernel events)
    nenc = max(1, args.enc_copies)
    copies = be.kind != "gpu" or (ncopy + nenc) * B * N <= 0.5 * be.free_bytes()
    # the timed encode rotates over nenc message buffers (same messages), so
    # no step re-encodes a buffer the Infinity Cache still holds
    enc = [cw]
    if copies:
        for _ in range(nenc - 1):
            b = be.like(cw)
            be.copy(b, clean)
            enc.append(b)
    bad = []
    if copies:  # one corrupted copy per step, made before the timed loop
        for _ in range(ncopy):
            b = be.like(cw)
            be.copy(b, clean)
            be.channel(b, err)
            bad.append(b)
        be.sync()

    def step(k):
        # the step's encode (messages in cw) and decode (a corrupted copy)
        # share no buffer: with --overlap the encode goes to a second stream
        be.encode(enc[k % len(enc)], side=args.overlap and copies and be.kind == "gpu")
        if copies:
            d = bad[k]
        else:
            be.channel(cw, err)
            d = cw
        be.decode(d, st)

    for k in range(args.warmup):
        step(k)
    # timed loop 1 (`value`): the codec kernels only
    ranks.barrier(be.sync)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    ranks.barrier(be.sync)
    elapsed = ranks.max(time.perf_counter() - t0)
    # timed loop 2: the same steps on fresh copies with HIP events on every
    # launch (poporon_amd_timing: hipExtLaunchKernel stamps them at the
    # kernel's own start and end, so they agree with a rocprofv3 kernel trace)
    # -- per-kernel times and the roofline; the events cost ~5 % of a step,
    # so they stay out of loop 1
    kt = None
    elapsed_ev = None
    if be.kind == "gpu" and copies:
        be.rs.timing(True)
        ranks.barrier(be.sync)
        t1 = time.perf_counter()
        for k in range(args.steps):
            step(args.warmup + args.steps + k)
        ranks.barrier(be.sync)
        elapsed_ev = ranks.max(time.perf_counter() - t1)
        kt = {k: be.rs.timing_read(k) for k in be.P.KERNEL_NAMES}
        be.rs.timing(False)
    nbad = be.n_bad(st, 16) + sum(be.n_diff(b, clean) for b in enc)
    timed = bad[args.warmup:args.warmup + (2 if elapsed_ev else 1) * args.steps] if copies else [cw]
    nbad += sum(be.n_diff(b, clean) for b in timed)
    # parity sample: every SAMPLE_STRIDE-th codeword's timed
    # encode and decode, checked against the reference after the timed loops
    idx = sample_index(B)
    rows = be.host(clean, idx)
    samples = {"encode": {"msg": rows[:, :K], "got_par": rows[:, K:], "first": first},
               "decode16": {"in": channel_rows(rows, be.host(err[0], idx), be.host(err[1], idx)),
                            "out": be.host(timed[-1], idx), "ok": be.host(st[0], idx), "cor": be.host(st[1], idx),
                            "first": first}}
    csum = be.checksum(cw, first)
    del bad, enc
    return {"elapsed": elapsed, "elapsed_ev": elapsed_ev, "kt": kt, "nbad": ranks.sum_int(nbad), "copies": copies,
            "checksum": ranks.sum_u64(csum), "cw": cw, "clean": clean, "err": err, "st": st, "samples": samples}


def run_erasure(be, ranks, args, rank, world, w, ne=32, nerr=0):
    """configs[3]: 32 sorted erasures per codeword in [0, 223), positions passed
    per codeword.  ne < 32 (the errata kernels): ne + nerr sorted unique
    positions in the message, every third one an error (not on the list),
    the rest the ne erasure slots; the stale slots past the count are 0, so
    the reference's slot-by-root-ordinal apply (src/decode.c:211-214) leaves
    these codewords changed, not restored: verified = ok and corrected_num
    (ne + nerr) for every codeword, the bytes by the GPU tests against the
    oracle (tests/test_gpu_split.py::test_errata_*)."""
    B = args.batch
    first = rank * B
    tot = ne + nerr
    pos, emag = be.errors(first, B, tot, K, SEED + 2 + (0 if ne == 32 else 7), sorted_positions=True)
    if nerr:
        keep = [k for k in range(tot) if k % 3 != 2][:ne] if nerr * 3 >= tot else list(range(ne))
        slots = be.torch.zeros((B, 32), dtype=be.torch.uint8, device=be.dev)
        slots[:, :ne] = pos[:, keep]
    else:
        slots = pos
    cnts = be.counts(B, ne)
    cw = w["cw"]
    be.encode(cw)
    eclean = be.like(cw)
    be.copy(eclean, cw)
    es = max(3, args.steps // 2)
    ecopies = (2 * es + 1) * B * N <= 0.5 * be.free_bytes()
    ebad = []
    if ecopies:
        for _ in range(2 * es + 1):
            b = be.like(cw)
            be.copy(b, eclean)
            be.channel(b, (pos, emag))
            ebad.append(b)

    def estep(k):
        if ecopies:
            d = ebad[k]
        else:
            be.channel(cw, (pos, emag))
            d = cw
        be.decode(d, w["st"], erasures=(slots, cnts))

    estep(0)
    # timed loop (cw_per_s): no per-kernel events; then the same decodes on
    # fresh copies with the events on (kernel times), as in run_weak
    ranks.barrier(be.sync)
    t0 = time.perf_counter()
    for k in range(es):
        estep(1 + k)
    ranks.barrier(be.sync)
    et = ranks.max(time.perf_counter() - t0)
    be.rs.timing(True)
    for k in range(es):
        estep(1 + es + k if ecopies else 0)
    be.sync()
    ekt = {k: be.rs.timing_read(k) for k in be.P.KERNEL_NAMES}
    ekt = {k: v for k, v in ekt.items() if v[1]}
    kms = sum(ms / es for ms, n in ekt.values())
    be.rs.timing(False)
    enbad = be.n_bad(w["st"], tot)
    if not nerr:
        enbad += sum(be.n_diff(b, eclean) for b in (ebad[1:] if ecopies else [cw]))
    enbad = ranks.sum_int(enbad)
    idx = sample_index(B)
    sample = {"in": channel_rows(be.host(eclean, idx), be.host(pos, idx), be.host(emag, idx)),
              "out": be.host(ebad[2 * es] if ecopies else cw, idx), "ok": be.host(w["st"][0], idx),
              "cor": be.host(w["st"][1], idx), "slots": be.host(slots, idx), "cnt": be.host(cnts, idx),
              "first": first}
    return {"cw_per_s": round(B * world * es / et, 1),
            "kernel_cw_per_s_per_gpu": round(B / (kms * 1e-3), 1) if kms else None,
            "kernels_avg_ms": {be.P.KERNEL_NAMES[k]: round(ms / n, 4) for k, (ms, n) in ekt.items()},
            "erasures": ne, "errors": nerr,
            "positions_bytes_per_cw": 32,
            "verified": enbad == 0,
            "channel": "outside the timed decodes (one corrupted copy per decode)" if ecopies
            else "in place, inside the timed decodes",
            "_kt": ekt, "_steps": es, "_sample": sample}


def mixed_counts(first, n):
    """Errors per codeword of the mixed channel: the binomial(255, MIXED_P)
    quantile of a counter hash of the global codeword index (so any sharding
    reproduces it), capped at MIXED_CAP."""
    import numpy as np
    from scipy.stats import binom

    import testutil as T
    h = T.synth_rows_cpu(SEED + 9, first, n, 4).astype(np.uint32)
    u = (h[:, 0] | (h[:, 1] << 8) | (h[:, 2] << 16) | (h[:, 3] << 24)).astype(np.float64)
    ne = binom.ppf((u + 0.5) / 4294967296.0, N, MIXED_P)
    return np.minimum(ne, MIXED_CAP).astype(np.uint8)


def run_mixed(be, ranks, args, rank, world, w):
    """A realistic channel: binomial(255, MIXED_P) errors per codeword, capped
    at MIXED_CAP (mean ~11.5; ~6-7 % of the codewords past t = 16, which the
    split kernels hand to the general kernel's list -- failures and the
    reference's miscorrections).  Codewords with <= 16 errors must come back
    restored with ok = 1 and corrected = their error count; every codeword's
    bytes, ok and count are in the parity sample against the reference."""
    B = args.batch
    first = rank * B
    ne_h = mixed_counts(first, B)
    pos, mag = be.errors(first, B, MIXED_CAP, N, SEED + 10)
    ne = be.from_host(ne_h)
    be.mask_errors(mag, ne)
    cw = w["clean"]
    es = max(3, args.steps // 2)
    mcopies = (2 * es + 1) * B * N <= 0.5 * be.free_bytes()
    mbad = []
    for _ in range(2 * es + 1 if mcopies else 1):
        b = be.like(cw)
        be.copy(b, cw)
        be.channel(b, (pos, mag))
        mbad.append(b)
    st = be.status(B)

    def mstep(k):
        if mcopies:
            d = mbad[k]
        else:
            be.copy(mbad[0], cw)
            be.channel(mbad[0], (pos, mag))
            d = mbad[0]
        be.decode(d, st)

    mstep(0)
    ranks.barrier(be.sync)
    gpu = be.kind == "gpu"
    t0 = time.perf_counter()
    for k in range(es):
        mstep(1 + k if mcopies else 0)
    ranks.barrier(be.sync)
    et = ranks.max(time.perf_counter() - t0)
    mkt = {}
    if gpu:  # kernel times from a second loop with the per-kernel events on
        be.rs.timing(True)
        for k in range(es):
            mstep(1 + es + k if mcopies else 0)
        be.sync()
        mkt = {k: be.rs.timing_read(k) for k in be.P.KERNEL_NAMES}
        mkt = {k: v for k, v in mkt.items() if v[1]}
        be.rs.timing(False)
    last = mbad[(2 * es if gpu else es)] if mcopies else mbad[0]
    nbad = ranks.sum_int(be.n_bad_mixed(st, ne, last, cw))
    idx = sample_index(B)
    sample = {"in": channel_rows(be.host(cw, idx), be.host(pos, idx), be.host(mag, idx)), "out": be.host(last, idx),
              "ok": be.host(st[0], idx), "cor": be.host(st[1], idx), "first": first}
    past = ranks.sum_int(int((ne_h > 16).sum()))
    okn = ranks.sum_int(be.count_ok(st))
    kms = sum(ms / es for ms, n in mkt.values())
    lst = mkt.get(be.P.KERNEL_LIST, (0.0, 0))[0] / es if gpu else 0.0
    return {"cw_per_s": round(B * world * es / et, 1),
            "kernel_cw_per_s_per_gpu": round(B / (kms * 1e-3), 1) if kms else None,
            "kernels_avg_ms": {be.P.KERNEL_NAMES[k]: round(ms / n, 4) for k, (ms, n) in mkt.items()} if gpu else {},
            "list_kernel_share": round(lst / kms, 4) if kms else None,
            "channel": f"binomial({N}, {MIXED_P}) errors per codeword (capped at {MIXED_CAP}), unique positions, "
                       "magnitudes in [1,255]",
            "mean_errors": round(float(ne_h.mean()), 3),
            "past_t_fraction": round(past / (B * world), 4),
            "ok_fraction": round(okn / (B * world), 4),
            "verified": nbad == 0,
            "_kt": mkt, "_steps": es, "_sample": sample}


# ----------------------------------------------------------------------------
# parity sample against the reference CPU path (SURVEY 8(d) "GPU timing")
# ----------------------------------------------------------------------------
SAMPLE_STRIDE = 4096
C4_SAMPLE_STRIDE = 65536  # configs[4]: 1,024 of the 2^26 codewords, whatever the split


def sample_index(B):
    import numpy as np
    return np.arange(0, B, SAMPLE_STRIDE, dtype=np.int64)


def channel_rows(rows, pos, mag):
    import numpy as np
    out = rows.copy()
    out[np.arange(rows.shape[0])[:, None], pos.astype(np.int64)] ^= mag
    return out


class ParityChecker:
    """The checker of the bench's parity sample: the reference itself
    (oracle/_ref/libpoporon_ref.so, libpoporon compiled from /root/reference/src,
    driven through its public single-codeword API: poporon_encode /
    poporon_decode, erasure lists via poporon_erasure_*) where it was built,
    else the clean-room restatement pinned to the reference's golden vectors
    (oracle/rs_oracle.c).  Runs after every timed loop; never on the codec path."""

    def __init__(self):
        from oracle import Oracle, Reference, reference_available
        self.kind = "reference" if reference_available() else "port"
        if self.kind == "reference":
            self.ref = Reference()
            self.eref = Reference(erasure=True)
        else:
            self.o = Oracle()

    def encode(self, msgs):
        import numpy as np
        if self.kind == "port":
            return self.o.encode_batch(msgs)
        return np.stack([self.ref.encode(m)[1] for m in msgs]) if len(msgs) else np.zeros((0, NR), np.uint8)

    def decode(self, rows, slots=None, cnt=None):
        """-> ok u8[n], corrected u8[n], rows' (data || parity) as the reference leaves them"""
        import numpy as np
        n = rows.shape[0]
        if self.kind == "port":
            if slots is None:
                ok, cor, d, p = self.o.decode_batch(rows[:, :K], rows[:, K:])
            else:
                ok, cor, d, p = self.o.decode_batch(rows[:, :K], rows[:, K:], slots.astype(np.uint32),
                                                    cnt.astype(np.uint32))
            return ok, cor.astype(np.uint8), np.concatenate([d, p], 1)
        ok, cor, out = np.zeros(n, np.uint8), np.zeros(n, np.uint8), rows.copy()
        for c in range(n):
            h = self.ref
            if slots is not None and int(slots[c].max()) >= K:
                # a slot past the message: the reference writes past the
                # caller's buffer there (quirk Q4, undefined) -- the pinned
                # restatement (which defines it) checks this row
                from oracle import Oracle
                r = Oracle().decode_batch(rows[c:c + 1, :K], rows[c:c + 1, K:], slots[c:c + 1].astype(np.uint32),
                                          cnt[c:c + 1].astype(np.uint32))
                r = (r[0][0], r[1][0], r[2][0], r[3][0])
                ok[c], cor[c] = r[0], r[1]
                out[c, :K], out[c, K:] = r[2], r[3]
                continue
            if slots is not None:
                h = self.eref
                # the batch API's slots past the count are the list's stale
                # entries of the reference (quirks Q1/Q2): fill all, then reset
                h.set_erasures(slots[c])
                h.set_erasures(slots[c][: int(cnt[c])])
            r = h.decode(rows[c, :K], rows[c, K:])
            ok[c], cor[c] = r[0], r[1]
            out[c, :K], out[c, K:] = r[2], r[3]
        return ok, cor, out

    def check(self, sm):
        """number of sampled codewords whose GPU result differs from the checker's"""
        import numpy as np
        if "msg" in sm:
            return int((self.encode(sm["msg"]) != sm["got_par"]).any(1).sum())
        ok, cor, out = self.decode(sm["in"], sm.get("slots"), sm.get("cnt"))
        bad = (ok != sm["ok"]) | (cor != sm["cor"]) | (out != sm["out"]).any(1)
        return int(bad.sum())


def parity_sample(samples, ranks):
    chk = ParityChecker()
    res = {"checker": ("reference: libpoporon compiled from /root/reference/src (oracle/_ref), public API"
                       if chk.kind == "reference" else
                       "port: clean-room restatement oracle/rs_oracle.c, pinned to the reference's golden vectors"),
           "stride": SAMPLE_STRIDE, "compares": "parity bytes (encode); decoded bytes, ok and corrected_num (decode)"}
    for mode, sm in samples.items():
        n = len(sm["msg"] if "msg" in sm else sm["in"])
        res[mode] = {"n": ranks.sum_int(n), "mismatches": ranks.sum_int(chk.check(sm))}
    return res


# ----------------------------------------------------------------------------
# rank-0 extras at N = 1
# ----------------------------------------------------------------------------
def host_pipeline(be, w, reps=3):
    """PCIe-inclusive rates of the host-memory batch API (poporon_encode_batch /
    poporon_decode_batch: pinned 3-slot pipeline) on the bench's own codewords,
    copied to host memory.  Reported beside `value`, never as it."""
    import ctypes as C

    import numpy as np
    rs, P = be.rs, be.P
    B = w["clean"].shape[0]
    host = w["clean"].cpu().numpy()
    msgs = np.ascontiguousarray(host[:, :K])
    par = np.zeros((B, NR), np.uint8)
    lib = rs.lib
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    te = []
    for _ in range(reps):
        t0 = time.perf_counter()
        assert lib.poporon_encode_batch(rs.h, vp(msgs), K, vp(par), NR, K, B), P.last_error()
        te.append(time.perf_counter() - t0)
    assert (par == host[:, K:]).all()
    bad = w["clean"].clone()
    be.channel(bad, w["err"])
    be.sync()
    bad = bad.cpu().numpy()
    ok = np.zeros(B, np.uint8)
    cor = np.zeros(B, np.uint8)
    td = []
    for _ in range(reps):
        work = bad.copy()
        t0 = time.perf_counter()
        assert lib.poporon_decode_batch(rs.h, vp(work), N, C.c_void_p(work.ctypes.data + K), N, K, B, None, 0, None,
                                        vp(ok), vp(cor)), P.last_error()
        td.append(time.perf_counter() - t0)
    assert ok.all() and (cor == 16).all() and (work == host).all()
    e, d = min(te), min(td)
    idx = np.arange(0, B, SAMPLE_STRIDE)  # the parity sample of this API's own outputs
    return {"encode_cw_per_s": round(B / e, 1), "encode_GB_per_s_pcie": round(B * (K + NR) / e / 1e9, 2),
            "decode_cw_per_s": round(B / d, 1), "decode_GB_per_s_pcie": round(B * (2 * N + 2) / d / 1e9, 2),
            "codewords": B, "note": "host-memory batch API, PCIe-inclusive (best of %d); not `value`" % reps,
            "_samples": {"host_encode": {"msg": msgs[idx], "got_par": par[idx]},
                         "host_decode16": {"in": bad[idx], "out": work[idx], "ok": ok[idx], "cor": cor[idx]}}}


def general_params(be, n=1 << 20, reps=5, params=(8, 0x11D, 1, 1, 16), nerr=8):
    """SURVEY 8(f) row 1, general parameters: RS(255, 239) -- the default field
    with 16 roots -- encode of n resident messages (the RS(255,223) LFSR kernel
    run with g(x) x^16, rsk_encode_nr) and decode with t = 8 random errors per
    codeword (the split kernels with npar = 16: rsk_syndrome_reset_nr,
    rs_bm_k<true>, Chien, Forney, rsk_apply_nr; the list on rs_generic.hip),
    wall time per call (stream-synchronised, median of reps).  Every 4096th codeword
    is compared with the oracle restatement (oracle/rs_oracle.c, pinned to the
    compiled reference's golden vectors for 13 parameter sets)."""
    import numpy as np

    from oracle import Oracle
    torch, P, T = be.torch, be.P, be.T
    m, poly, fcr, prim, nr = params
    k = 255 - nr
    h = P.Poporon(m, poly, fcr, prim, nr, device=be.local)
    s = be.stream
    rows = torch.empty((n, N), dtype=torch.uint8, device=be.dev)
    T.synth_rows(SEED + 40, 0, n, k, rows.data_ptr(), N, s)
    b = rows.data_ptr()
    h.encode_batch_device(b, N, b + k, N, k, n, s)  # warm-up
    te = []
    for _ in range(reps):
        be.sync()
        t0 = time.perf_counter()
        h.encode_batch_device(b, N, b + k, N, k, n, s)
        be.sync()
        te.append(time.perf_counter() - t0)
    clean = rows.clone()
    pos, mag = be.errors(0, n, nerr, N, SEED + 41)
    bad = clean.clone()
    T.channel_xor(pos.data_ptr(), mag.data_ptr(), nerr, bad.data_ptr(), N, n, s)
    ok, cor = be.status(n)
    td = []
    for r in range(reps + 1):
        rows.copy_(bad)
        be.sync()
        t0 = time.perf_counter()
        h.decode_batch_device(b, N, b + k, N, k, n, ok.data_ptr(), cor.data_ptr(), stream=s)
        be.sync()
        if r:
            td.append(time.perf_counter() - t0)
    nbad = be.n_bad((ok, cor), nerr) + be.n_diff(rows, clean)
    # one more decode with the kernel events on: where the time goes
    rows.copy_(bad)
    be.sync()
    h.timing(True)
    h.decode_batch_device(b, N, b + k, N, k, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    be.sync()
    kms = {}
    for kid, name in P.KERNEL_NAMES.items():
        ms, cnt = h.timing_read(kid)
        if cnt:  # (the hand-off list of a code with < 32 roots runs on the general kernel)
            kms[name.replace("rs_wave_k (list)", "rsgw_decode_k (list)")] = round(ms / cnt, 4)
    h.timing(False)
    nbad += be.n_bad((ok, cor), nerr) + be.n_diff(rows, clean)
    idx = sample_index(n)
    got, gok, gcor = be.host(rows, idx), be.host(ok, idx), be.host(cor, idx)  # the error decode's sample
    # erasure decode: nr sorted erasure slots in the data per codeword (the
    # configs[3] shape for this code), u8 slots at stride nr
    epos, emag = be.errors(0, n, nr, k, SEED + 42, sorted_positions=True)
    ebad = clean.clone()
    T.channel_xor(epos.data_ptr(), emag.data_ptr(), nr, ebad.data_ptr(), N, n, s)
    ecnt = be.counts(n, nr)
    tx = []
    for r in range(reps + 1):
        rows.copy_(ebad)
        be.sync()
        t0 = time.perf_counter()
        h.decode_batch_device(b, N, b + k, N, k, n, ok.data_ptr(), cor.data_ptr(), d_positions=epos.data_ptr(),
                              positions_stride=nr, d_counts=ecnt.data_ptr(), stream=s)
        be.sync()
        if r:
            tx.append(time.perf_counter() - t0)
    nbad += be.n_bad((ok, cor), nr) + be.n_diff(rows, clean)
    o = Oracle(*params)
    smp_clean, smp_bad = be.host(clean, idx), be.host(bad, idx)
    mism = int((o.encode_batch(smp_clean[:, :k]) != smp_clean[:, k:]).any(1).sum())
    ook, ocor, od, op = o.decode_batch(smp_bad[:, :k], smp_bad[:, k:])
    mism += int(((ook != gok) | (ocor != gcor) | (od != got[:, :k]).any(1) | (op != got[:, k:]).any(1)).sum())
    smp_ebad, smp_slots = be.host(ebad, idx), be.host(epos, idx)
    xok, xcor, xd, xp = o.decode_batch(smp_ebad[:, :k], smp_ebad[:, k:], smp_slots.astype(np.uint32),
                                       np.full(len(idx), nr, np.uint32))
    got = be.host(rows, idx)
    xgok, xgcor = be.host(ok, idx), be.host(cor, idx)
    mism += int(((xok != xgok) | (xcor != xgcor) | (xd != got[:, :k]).any(1) | (xp != got[:, k:]).any(1)).sum())
    e, d, x = float(np.median(te)), float(np.median(td)), float(np.median(tx))
    h.close()
    return {"code": f"RS(255,{k}): symbol_size {m}, poly {poly:#x}, fcr {fcr}, prim {prim}, {nr} roots",
            "kernels": "encode: rs_lfsr_k<ENCODE> with g(x) x^(32 - nr) (rsk_encode_nr); decode: the split "
                       "kernels with npar = nr (rsk_syndrome_reset_nr, rs_bm_k<true>, rs_chien_k, rs_forney_k, "
                       "rsk_apply_nr; hand-off list on rsgw_decode_k); erasure decode: the errata kernels with npar "
                       "= nr (rsk_ebm_nr, rs_chien32_k, rsk_forney32_nr, rsk_apply_era_nr)", "codewords": n,
            "errors_per_codeword": nerr,
            "encode_cw_per_s": round(n / e, 1), "decode_cw_per_s": round(n / d, 1),
            "encode_ms": round(e * 1e3, 4), "decode_ms": round(d * 1e3, 4), "decode_kernels_ms": kms,
            "erasure_decode_cw_per_s": round(n / x, 1), "erasure_decode_ms": round(x * 1e3, 4),
            "erasures_per_codeword": nr,
            "hbm_frac_encode": round(n * N / e / 1e9 / HBM_PEAK_GBS, 4),
            "hbm_frac_decode": round(n * N / d / 1e9 / HBM_PEAK_GBS, 4),
            "timing": f"wall time per call, stream-synchronised, median of {reps}",
            "verified": nbad == 0 and mism == 0,
            "sample": {"checker": "port: oracle/rs_oracle.c (pinned)", "n": int(len(idx)), "mismatches": mism}}


def general_wave(be, sets=((8, 0x11D, 1, 1, 100), (4, 0x13, 1, 2, 8)), n=1 << 16, calls=200, reps=7):
    """SURVEY 8(f) row 1 beyond the fewer-roots codes: parameter sets of the
    reference's own tests that run on the general kernels (rs_generic.hip) --
    RS(255,155) (100 roots: decode one codeword per wave, two per pass,
    rsgw_*; batch encode on the per-lane LFSR rsg_lfsr_k) and RS(15,7) over
    GF(16) with prim 2 (decode sixteen codewords per wave, 4-lane groups;
    batch encode on the RS(255,223) LFSR kernel): single-call encode / decode
    latency through ctypes (t errors), a device batch decode of n codewords
    with t errors each (wall, stream-synchronised, and device events; median
    of reps) and a device batch encode (device events).  Every 256th batch
    codeword and every single call are compared with the oracle restatement."""
    import numpy as np

    from oracle import Oracle
    torch, P = be.torch, be.P
    s = be.stream
    out = {}
    for params in sets:
        m, poly, fcr, prim, nr = params
        nn = (1 << m) - 1
        k, t = nn - nr, nr // 2
        h, o = P.Poporon(*params, device=be.local), Oracle(*params)
        rng = np.random.default_rng(SEED + nr + m)
        data = rng.integers(0, nn + 1, (n, k), dtype=np.uint8)
        par = h.encode_batch(data)
        mism = int((par[::256] != o.encode_batch(data[::256])).any(1).sum())
        cw = np.concatenate([data, par], 1)
        pos = np.argsort(rng.random((n, nn)), axis=1)[:, :t]
        bad = cw.copy()
        np.bitwise_xor.at(bad, (np.arange(n)[:, None], pos), rng.integers(1, nn + 1, (n, t), dtype=np.uint8))
        # single calls
        h.encode(data[0])
        t0 = time.perf_counter()
        spar = [h.encode(data[i]) for i in range(calls)]
        te = (time.perf_counter() - t0) / calls
        mism += sum(int((spar[i] != par[i]).any()) for i in range(calls))
        h.decode(bad[0, :k], bad[0, k:])
        t0 = time.perf_counter()
        res = [h.decode(bad[i, :k], bad[i, k:]) for i in range(calls)]
        td = (time.perf_counter() - t0) / calls
        for i in range(calls):
            wok, wn, wd, wp = o.decode(bad[i, :k], bad[i, k:])
            mism += int(res[i][0] != wok or res[i][1] != wn or (res[i][2] != wd).any() or (res[i][3] != wp).any())
        # device batch
        src = torch.from_numpy(bad).to(be.dev)
        buf = src.clone()
        ok, cor = be.status(n)
        b = buf.data_ptr()
        tb, tk = [], []
        for r in range(reps + 1):
            buf.copy_(src)
            be.sync()
            t0 = time.perf_counter()
            h.decode_batch_device(b, nn, b + k, nn, k, n, ok.data_ptr(), cor.data_ptr(), stream=s)
            be.sync()
            if r:
                tb.append(time.perf_counter() - t0)
        for r in range(reps):  # device time: the stream kept busy while the host enqueues (no launch gap counted)
            buf.copy_(src)
            be.sync()
            torch.cuda._sleep(200000)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.decode_batch_device(b, nn, b + k, nn, k, n, ok.data_ptr(), cor.data_ptr(), stream=s)
            e1.record()
            be.sync()
            tk.append(e0.elapsed_time(e1) * 1e-3)
        got, gok, gcor = buf.cpu().numpy(), ok.cpu().numpy(), cor.cpu().numpy()
        # device batch encode of the same messages into rows [data | parity]
        erow = torch.from_numpy(np.concatenate([data, np.zeros_like(par)], 1)).to(be.dev)
        eb = erow.data_ptr()
        te_dev = []
        for r in range(reps + 1):
            be.sync()
            torch.cuda._sleep(200000)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.encode_batch_device(eb, nn, eb + k, nn, k, n, s)
            e1.record()
            be.sync()
            if r:
                te_dev.append(e0.elapsed_time(e1) * 1e-3)
        mism += int((erow.cpu().numpy()[:, k:] != par).any(1).sum())
        idx = np.arange(0, n, 256)
        ook, ocor, od, op = o.decode_batch(bad[idx, :k], bad[idx, k:])
        mism += int(((ook != gok[idx]) | (ocor != gcor[idx]) | (od != got[idx, :k]).any(1) |
                     (op != got[idx, k:]).any(1)).sum())
        mism += int((got != cw).any(1).sum())  # t errors: every codeword back to the encoded row
        d, dk = float(np.median(tb)), float(np.median(tk))
        out[f"RS({nn},{k})"] = {
            "params": {"symbol_size": m, "poly": hex(poly), "fcr": fcr, "prim": prim, "num_roots": nr},
            "single_encode_us": round(te * 1e6, 1), "single_decode_us": round(td * 1e6, 1),
            "batch_codewords": n, "batch_decode_cw_per_s": round(n / d, 1), "batch_decode_ms": round(d * 1e3, 4),
            "batch_decode_device_cw_per_s": round(n / dk, 1), "batch_decode_device_ms": round(dk * 1e3, 4),
            "batch_encode_device_cw_per_s": round(n / float(np.median(te_dev)), 1),
            "batch_encode_device_ms": round(float(np.median(te_dev)) * 1e3, 4),
            "errors_per_codeword": t, "mismatches": mism}
        h.close()
    out["note"] = ("single calls: poporon_encode / poporon_decode through ctypes (one wave, coherent host memory); "
                   "batch: poporon_decode_batch_device, wall time of the Python call (batch_decode_*) and device "
                   "time between HIP events on its stream (batch_decode_device_*); poporon_encode_batch_device of the "
                   "same messages (batch_encode_device_*, its parity equal to the host batch's, which is sampled "
                   "against the oracle); checked against oracle/rs_oracle.c")
    out["verified"] = all(v["mismatches"] == 0 for kk, v in out.items() if isinstance(v, dict))
    return out


def call_latency(be, calls=2000):
    """The reference's calling pattern: one codeword per poporon_encode /
    poporon_decode call (include/poporon.h:90-91), host buffers, on the GPU
    (the single-call server rs_serve_k).  Timed by a C loop through the
    library's own entry points (testutil ptu_time_encode / ptu_time_decode),
    as the CPU baseline's C loop times the reference; the same calls made
    one by one from Python through ctypes are reported beside it."""
    import ctypes as C

    import numpy as np

    import testutil as T
    rs = be.rs
    lib = rs.lib
    msgs = T.synth_rows_cpu(SEED + 7, 0, calls, K)
    pos, mag = T.synth_errors_cpu(SEED + 8, 0, calls, 16, N)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    par = np.zeros((calls, NR), np.uint8)
    for c in range(16):  # warm-up (staging allocation, the server's first launch)
        lib.poporon_encode(rs.h, vp(msgs[c]), K, vp(par[c]))
    te = T.time_encode(lib, rs.h, msgs, par)
    cw = T.channel_xor_cpu(np.concatenate([msgs, par], 1), pos, mag)
    d, p = np.ascontiguousarray(cw[:, :K]), np.ascontiguousarray(cw[:, K:])
    td, ok, cor = T.time_decode(lib, rs.h, d, p)
    assert te > 0 and ok.all() and (cor == 16).all() and (d == msgs).all()
    # the same through ctypes, one Python call each
    par2 = np.zeros((calls, NR), np.uint8)
    t0 = time.perf_counter()
    for c in range(calls):
        lib.poporon_encode(rs.h, vp(msgs[c]), K, vp(par2[c]))
    tpe = time.perf_counter() - t0
    d2, p2 = np.ascontiguousarray(cw[:, :K]), np.ascontiguousarray(cw[:, K:])
    n = C.c_size_t(0)
    fixed = 0
    t0 = time.perf_counter()
    for c in range(calls):
        fixed += bool(lib.poporon_decode(rs.h, vp(d2[c]), K, vp(p2[c]), C.byref(n))) and n.value == 16
    tpd = time.perf_counter() - t0
    assert (par2 == par).all() and fixed == calls and (d2 == msgs).all()
    return {"encode_us_per_call": round(te / calls * 1e6, 2), "decode16_us_per_call": round(td / calls * 1e6, 2),
            "python_ctypes_encode_us_per_call": round(tpe / calls * 1e6, 2),
            "python_ctypes_decode16_us_per_call": round(tpd / calls * 1e6, 2),
            "calls": calls, "note": "poporon_encode / poporon_decode (16 errors), one codeword per call, host buffers, "
                                    "a C loop (as cpu_baseline's T1 loop of the reference); python_ctypes_*: the same "
                                    "calls from a Python loop"}


def _cpu_info():
    model, host = "unknown", os.cpu_count() or 1
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = host
    quota = None
    try:  # cgroup v2 CPU quota ("max 100000" = none)
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    usable = min(avail, quota) if quota else avail
    return model, host, avail, quota, usable


def cpu_baseline(seconds_target=6.0):
    """The reference CPU path (oracle/_ref: libpoporon compiled from
    /root/reference/src/*.c, AVX2 build) through its public single-codeword
    API, one handle per thread over contiguous slices (oracle/ref_harness.c),
    at T = 1 and T = every core this process may use; encode and 16-error
    decode timed separately on a bounded sample.  Falls back to the clean-room
    restatement (oracle/rs_oracle.c, bit-identical) where _ref is absent."""
    import ctypes as C

    import numpy as np

    import testutil as T
    from oracle import HERE as OR_DIR, Oracle
    model, host, avail, quota, usable = _cpu_info()
    ref_so = os.path.join(OR_DIR, "_ref", "libpoporon_refbench.so")
    o = Oracle()
    if os.path.exists(ref_so):
        lib = C.CDLL(ref_so)
        kind, label = "reference", "libpoporon (AVX2 build of /root/reference/src) via its public API"

        def enc(d, p, t):
            lib.refbench_encode(d.ctypes.data_as(C.c_void_p), C.c_size_t(K), p.ctypes.data_as(C.c_void_p),
                                C.c_size_t(NR), C.c_size_t(K), C.c_size_t(d.shape[0]), C.c_int(t))

        def dec(d, p, ok, cor, t):
            lib.refbench_decode(d.ctypes.data_as(C.c_void_p), C.c_size_t(K), p.ctypes.data_as(C.c_void_p),
                                C.c_size_t(NR), C.c_size_t(K), C.c_size_t(d.shape[0]), ok.ctypes.data_as(C.c_void_p),
                                cor.ctypes.data_as(C.c_void_p), C.c_int(t))
    else:
        kind, label = "port", "clean-room C restatement (oracle/rs_oracle.c), bit-identical to the reference"

        def enc(d, p, t):
            p[:] = o.encode_batch(d, threads=t)

        def dec(d, p, ok, cor, t):
            r = o.decode_batch(d, p, threads=t)
            ok[:], cor[:] = r[0], r[1]
            d[:], p[:] = r[2], r[3]

    def rates(n, t):
        d = T.synth_rows_cpu(SEED, 0, n, K)
        p = np.zeros((n, NR), np.uint8)
        t0 = time.perf_counter()
        enc(d, p, t)
        te = time.perf_counter() - t0
        assert (p[:64] == o.encode_batch(d[:64])).all()
        pos, mag = T.synth_errors_cpu(SEED + 1, 0, n, 16, N)
        cw = T.channel_xor_cpu(np.concatenate([d, p], 1), pos, mag)
        d2, p2 = np.ascontiguousarray(cw[:, :K]), np.ascontiguousarray(cw[:, K:])
        ok, cor = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        t0 = time.perf_counter()
        dec(d2, p2, ok, cor, t)
        td = time.perf_counter() - t0
        assert ok.all() and (cor == 16).all() and (d2 == d).all()
        return n / te, n / td

    out = {}
    for t in sorted({1, usable}):
        e0, d0 = rates(256 * t, t)  # calibration
        n = int(max(512 * t, min(1 << 20, seconds_target / 2 / (1 / e0 + 1 / d0))))
        e, d = rates(n, t)
        out[t] = (e, d, n)
    e, d, n = out[usable]
    e1, d1, n1 = out[1]
    return {"value": round(1.0 / (1.0 / e + 1.0 / d), 1), "unit": "codewords/s", "cores": usable, "kind": kind,
            "sample": f"{n} codewords at T={usable} ({n1} at T=1): encode, then 16-error decode, one handle per "
                      f"thread, {label}",
            "value_def": "round trips/s = 1 / (1/encode + 1/decode) at T=cores",
            "cpu_model": model, "host_logical_cpus": host, "affinity_cpus": avail, "cgroup_cpu_quota": quota,
            "T1": {"encode_cw_per_s": round(e1, 1), "decode16_cw_per_s": round(d1, 1),
                   "encode_us_per_cw": round(1e6 / e1, 2), "decode16_us_per_cw": round(1e6 / d1, 2)},
            "Tall": {"threads": usable, "encode_cw_per_s": round(e, 1), "decode16_cw_per_s": round(d, 1)}}


# ----------------------------------------------------------------------------
def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    rc = launch_ranks(args, argv)
    if rc is not None:
        sys.exit(rc)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")

    if args.backend:
        mod = importlib.import_module(args.backend)
        world, rank, local = dist_setup(mod.Backend.dist_backend)
        be = mod.Backend(local)
        dev = "cpu"
    else:
        world, rank, local = dist_setup("nccl")
        be = GpuBackend(local)
        dev = "cpu" if one_device() else be.dev
    ranks = Ranks(world, dev)

    w = run_weak(be, ranks, args, rank, world)
    gpu = be.kind == "gpu"
    B = args.batch
    elapsed = w["elapsed"]
    value = B * world * args.steps / elapsed
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "ms_per_step_instrumented": (round(w["elapsed_ev"] / args.steps * 1e3, 4) if w.get("elapsed_ev") else None),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-hash messages, 16 random-magnitude errors at unique positions per codeword)",
        "config": {"workload": "RS(255,223) round trip: encode + decode with 16 errors per codeword, "
                               f"{B} codewords per GPU (BASELINE configs[1]+[2]); configs[4] (the "
                               f"{args.c4_total}-codeword strong split) under 'configs4'",
                   "codewords_per_gpu": B, "layout": "255-byte codeword rows, stride 255",
                   "code": "poporon_config_rs_default (8, 0x11D, fcr 1, prim 1, 32 roots)"},
        # one bandwidth definition everywhere: 255 B per codeword
        # per mode, so a round trip (encode + decode) counts 510 B
        "GB_per_s": round(value * 2 * CW_BYTES / 1e9, 2),
        "hbm_frac_of_peak": round(value * 2 * CW_BYTES / 1e9 / (HBM_PEAK_GBS * world), 4),
        "bytes_per_unit": "510 = 255 (encode: 223 read + 32 written) + 255 (decode: 255 read) per round trip",
        "step": f"encode {B} messages + decode {B} corrupted codewords (16 errors each); the test channel corrupts "
                "one copy per step before the timed loops; `value` / `ms_per_step` from a loop without per-kernel "
                "events, per-kernel times and the roofline from a second loop of the same steps with HIP events "
                "stamped by every kernel's dispatch (`ms_per_step_instrumented`)" if w["copies"]
                else "encode + channel (in place) + decode",
        "verified": w["nbad"] == 0,
        "weak_checksum": w["checksum"],
    }
    if one_device() and not args.backend:
        line["rehearsal"] = f"POPORON_BENCH_ONE_DEVICE: all {world} ranks on cuda:0, gloo reductions; not a scaling number"
    samples = dict(w.pop("samples"))
    if not args.no_mixed:
        mix = run_mixed(be, ranks, args, rank, world, w)
        samples["decode_mixed"] = mix.pop("_sample")
        line["decode_mixed"] = mix
        line["verified"] = line["verified"] and mix["verified"]
    if gpu and w["kt"]:
        P = be.P
        kt = {k: v for k, v in w["kt"].items() if v[1]}
        per_kernel = {}
        # a kernel may run several times per step (the split decode works in
        # sub-batches): per-step time = total / steps, codewords per launch =
        # B * steps / launches.  No per-kernel GB/s: the 255 algorithmic bytes
        # belong to a mode's whole path, not to one of its stages.
        step_ms = {k: ms / args.steps for k, (ms, n) in kt.items()}
        avg_ms = {k: ms / n for k, (ms, n) in kt.items()}
        per_launch = {k: B * args.steps / n for k, (ms, n) in kt.items()}
        traffic, tnote = load_traffic(args.traffic)
        for k, (ms, n) in kt.items():
            per_kernel[P.KERNEL_NAMES[k]] = {"ms_per_step": round(step_ms[k], 4), "avg_ms": round(avg_ms[k], 4),
                                             "launches": n, "codewords_per_launch": int(per_launch[k]),
                                             "cw_per_s_per_gpu": round(B / (step_ms[k] * 1e-3), 1)}
        if world > 1:  # every rank's kernel times (the line's other kernel figures are rank 0's)
            ids = sorted(P.KERNEL_NAMES)
            allr = ranks.gather([w["kt"].get(k, (0.0, 0))[0] / args.steps for k in ids], ranks.torch.float64)
            line["kernels_per_rank_ms_per_step"] = {P.KERNEL_NAMES[k]: [round(r[i], 4) for r in allr]
                                                    for i, k in enumerate(ids) if any(r[i] for r in allr)}
        enc_ms = sum(v for k, v in step_ms.items() if k == P.KERNEL_ENCODE)
        dec_ms = sum(v for k, v in step_ms.items() if k != P.KERNEL_ENCODE)
        modes = {"encode": path_roofline("encode", kt, args.steps, B, traffic),
                 "decode16": path_roofline("decode16", kt, args.steps, B, traffic)}
        if not args.no_erasure:
            era = run_erasure(be, ranks, args, rank, world, w)
            modes["erasure32"] = path_roofline("erasure32", era.pop("_kt"), era.pop("_steps"), B, traffic)
            samples["erasure32"] = era.pop("_sample")
            line["erasure_decode_32"] = era
            eta = run_erasure(be, ranks, args, rank, world, w, ne=16, nerr=8)
            modes["errata16e8"] = path_roofline("errata16e8", eta.pop("_kt"), eta.pop("_steps"), B, traffic)
            samples["errata16e8"] = eta.pop("_sample")
            line["errata_decode_16e8"] = eta
            line["verified"] = line["verified"] and era["verified"] and eta["verified"]
        if "decode_mixed" in line:
            modes["decode_mixed"] = path_roofline("decode_mixed", line["decode_mixed"].pop("_kt"),
                                                  line["decode_mixed"].pop("_steps"), B, traffic)
        if modes["encode"] and modes["decode16"]:
            rt_ms = modes["encode"]["path_ms"] + modes["decode16"]["path_ms"]
            rt = 2 * B * CW_BYTES / (rt_ms * 1e-3) / 1e9
            modes["roundtrip"] = {"achieved": round(rt, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(rt / HBM_PEAK_GBS, 4), "path_ms": round(rt_ms, 4),
                                  "algorithmic_bytes": 2 * B * CW_BYTES,
                                  "traffic": (modes["encode"]["traffic"] + modes["decode16"]["traffic"]
                                              if modes["encode"]["traffic"] and modes["decode16"]["traffic"]
                                              else None),
                                  "note": "encode path + decode16 path, 255 B per codeword per mode"}
        modes = {k: v for k, v in modes.items() if v}
        roof = dict(modes.get("decode16") or {})
        roof.update({"kernel": "decode16 path (" + " + ".join(P.KERNEL_NAMES[k] for k in roof.get("kernels_ms", {}))
                               + ")",
                     "note": "path-level: 255 B x codewords / sum of the path's kernel times per step (HIP events "
                             "stamped by each kernel's dispatch, hipExtLaunchKernel); traffic = HBM bytes of the same path from rocprofv3 "
                             "FETCH_SIZE x 2 + WRITE_SIZE (tools/pmc_traffic.py); the kernels are VALU/LDS-bound, "
                             "see DESIGN.md"})
        roof["kernels_ms"] = {P.KERNEL_NAMES[k]: v for k, v in roof.get("kernels_ms", {}).items()}
        for m in modes.values():
            if "kernels_ms" in m:
                m["kernels_ms"] = {P.KERNEL_NAMES.get(k, k): v for k, v in m["kernels_ms"].items()}
        line.update({
            "encode_cw_per_s_per_gpu": round(B / (enc_ms * 1e-3), 1),
            "decode_cw_per_s_per_gpu": round(B / (dec_ms * 1e-3), 1),
            "kernels": per_kernel,
            "roofline": roof,
            "roofline_modes": modes,
            "traffic_source": (f"{args.traffic} (stamp {traffic.get('source_stamp')}, measured {traffic.get('date')})"
                               if traffic else tnote),
        })
        if world == 1 and not args.no_host:
            hp = host_pipeline(be, w)
            samples.update(hp.pop("_samples"))
            line["host_pipeline"] = hp
        if world == 1 and not args.no_latency:
            line["single_call_latency"] = call_latency(be)
        if world == 1 and not args.no_general:
            gp = general_params(be)
            line["general_params"] = gp
            line["verified"] = line["verified"] and gp["verified"]
            gw = general_wave(be)
            line["general_wave"] = gw
            line["verified"] = line["verified"] and gw["verified"]
    else:
        if "decode_mixed" in line:
            line["decode_mixed"].pop("_kt", None)
            line["decode_mixed"].pop("_steps", None)
    del w
    if not args.no_c4:
        c4 = run_strong(be, ranks, args, rank, world)
        samples.update(c4.pop("_samples"))
        line["configs4"] = c4
        line["parity_checksum"] = c4["parity_checksum"]
        line["verified"] = line["verified"] and c4["verified"]
    if args.c4_scatter and world > 1:
        sc = run_scatter(be, ranks, args, rank, world)
        line["configs4_scatter"] = sc
        line["verified"] = line["verified"] and sc["verified"]
    # every sampled codeword of every mode against the reference CPU path
    # (after all timed loops)
    ps = parity_sample(samples, ranks)
    line["parity_sample"] = ps
    line["verified"] = line["verified"] and all(v["mismatches"] == 0 for k, v in ps.items() if isinstance(v, dict))
    if gpu and rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
        lat = line.get("single_call_latency")
        if lat:  # the drop-in path against the reference on one host core, same box and run
            t1 = line["cpu_baseline"]["T1"]
            lat["vs_reference_T1"] = {"encode": round(t1["encode_us_per_cw"] / lat["encode_us_per_call"], 3),
                                      "decode16": round(t1["decode16_us_per_cw"] / lat["decode16_us_per_call"], 3),
                                      "note": "> 1: the GPU call is faster than the reference's call on one core"}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
