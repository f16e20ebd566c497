#!/usr/bin/env python3
"""bench.py -- RS(255,223) encode + decode@16 throughput on MI355X.

One step = one pass of the hot path over one batch of synthetic codewords
resident in HBM (configs[1] + configs[2] of BASELINE.json, chained):

    encode  2^20 messages x 223 B -> 32 parity bytes each        (HIP, C ABI)
    decode  2^20 codewords with 16 errors each (unique positions over all 255
            bytes, magnitudes in [1,255]): remainder + syndromes/BM/Chien/
            Forney/apply, in place                               (HIP, C ABI)

The errors come from the test channel (csrc/channel.hip), which is not part of
the codec: before the timed loop it corrupts one copy of the encoded batch per
step, and step k decodes copy k, so every step does the full decode work and
the timed loop holds only codec kernels.  (The round-1 shape -- channel inside
the step, decode in place -- is timed too and reported as
roundtrip_with_channel_cw_per_s.)  Codeword layout: one 255-byte row per
codeword (data then parity), stride 255.  value = codewords through encode +
decode per second, summed over all ranks (weak scaling: 2^20 codewords per
GPU).  Inputs are generated on the device from a counter-based hash of (seed,
global codeword index), so any sharding sees the same codewords.

Multi-GPU: launched by torch.distributed.run, one process per GPU; the
codeword range is split across ranks with no data-path collective (RCCL only
for the barrier and the max-time / verification reductions).

Also reported: per-kernel HIP-event times (in-library, on the launch
stream), the roofline of the dominant kernel, erasure decode (configs[3]),
and the reference CPU path timed on the host cores (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import libpoporon_amd as P  # noqa: E402

METRIC = "RS(255,223) codewords/s (encode; decode @ t=16 errs) and GB/s vs HBM peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CW_BYTES = 255         # algorithmic bytes per codeword
K, NR, N = 223, 32, 255
SEED = 0x5EED0001


# ----------------------------------------------------------------------------
# counter-based synthetic data (murmur3 fmix32 of (seed, counter)) on device
# ----------------------------------------------------------------------------
def _fmix32(x):
    M = 0xFFFFFFFF
    x = x & M
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & M
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & M
    return x ^ (x >> 16)


def synth_bytes(seed, first, count, width, device):
    """uint8 [count, width]: byte j of row i = hash(seed, (first+i)*width + j)."""
    out = torch.empty((count, width), dtype=torch.uint8, device=device)
    step = max(1, (1 << 24) // width)
    cols = torch.arange(width, device=device, dtype=torch.int64)
    for a in range(0, count, step):
        b = min(count, a + step)
        rows = torch.arange(first + a, first + b, device=device, dtype=torch.int64)
        ctr = rows[:, None] * width + cols[None, :]
        out[a:b] = (_fmix32(ctr * 0x9E3779B1 + seed) & 0xFF).to(torch.uint8)
    return out


def synth_errors(seed, first, count, nerr, span, device):
    """nerr unique positions in [0, span) and magnitudes in [1,255] per row."""
    pos = torch.empty((count, nerr), dtype=torch.int64, device=device)
    mag = torch.empty((count, nerr), dtype=torch.uint8, device=device)
    step = max(1, (1 << 24) // span)
    cols = torch.arange(span, device=device, dtype=torch.int64)
    for a in range(0, count, step):
        b = min(count, a + step)
        rows = torch.arange(first + a, first + b, device=device, dtype=torch.int64)
        keys = _fmix32((rows[:, None] * span + cols[None, :]) * 0x9E3779B1 + seed)
        pos[a:b] = keys.topk(nerr, dim=1).indices
        m = _fmix32((rows[:, None] * nerr + cols[None, :nerr]) * 0x9E3779B1 + seed + 0x1234567)
        mag[a:b] = (m % 255 + 1).to(torch.uint8)
    return pos, mag


# ----------------------------------------------------------------------------
def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def allreduce(x, op, world, device="cuda"):
    """Scalar reduction over ranks (RCCL on GPU, gloo on CPU in the tests)."""
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=op)
    return float(t.item())


def cpu_baseline(seconds_target=8.0):
    """The reference CPU path (oracle/_ref, built from /root/reference/src),
    one handle per thread over contiguous slices, timed on this host."""
    import ctypes as C

    from oracle import HERE as OR_DIR, Oracle
    ref_so = os.path.join(OR_DIR, "_ref", "libpoporon_refbench.so")
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))
    o = Oracle()
    rng = np.random.default_rng(SEED)

    def make(n):
        data = rng.integers(0, 256, (n, K), dtype=np.uint8)
        par = np.zeros((n, NR), np.uint8)
        return data, par

    if os.path.exists(ref_so):
        lib = C.CDLL(ref_so)
        kind, label = "reference", "libpoporon (AVX2 build of /root/reference/src) via its public API"

        def enc(d, p):
            lib.refbench_encode(d.ctypes.data_as(C.c_void_p), C.c_size_t(K), p.ctypes.data_as(C.c_void_p),
                                C.c_size_t(NR), C.c_size_t(K), C.c_size_t(d.shape[0]), C.c_int(threads))

        def dec(d, p, ok, cor):
            lib.refbench_decode(d.ctypes.data_as(C.c_void_p), C.c_size_t(K), p.ctypes.data_as(C.c_void_p),
                                C.c_size_t(NR), C.c_size_t(K), C.c_size_t(d.shape[0]), ok.ctypes.data_as(C.c_void_p),
                                cor.ctypes.data_as(C.c_void_p), C.c_int(threads))
    else:
        kind, label = "port", "clean-room C restatement (oracle/rs_oracle.c), bit-identical to the reference"

        def enc(d, p):
            p[:] = o.encode_batch(d, threads=threads)

        def dec(d, p, ok, cor):
            r = o.decode_batch(d, p, threads=threads)
            ok[:], cor[:] = r[0], r[1]
            d[:], p[:] = r[2], r[3]

    def roundtrip(n):
        d, p = make(n)
        t0 = time.perf_counter()
        enc(d, p)
        t1 = time.perf_counter()
        cw = np.concatenate([d, p], 1)
        for a in range(0, n, 65536):
            b = min(n, a + 65536)
            pos = np.argpartition(rng.random((b - a, N), dtype=np.float32), 16, axis=1)[:, :16]
            rows = np.arange(a, b)[:, None]
            cw[rows, pos] ^= rng.integers(1, 256, (b - a, 16), dtype=np.uint8)
        d2, p2 = np.ascontiguousarray(cw[:, :K]), np.ascontiguousarray(cw[:, K:])
        ok = np.zeros(n, np.uint8)
        cor = np.zeros(n, np.uint8)
        t2 = time.perf_counter()
        dec(d2, p2, ok, cor)
        t3 = time.perf_counter()
        assert ok.all() and (cor == 16).all() and (d2 == d).all()
        return (t1 - t0), (t3 - t2)

    te, td = roundtrip(2048 * threads)
    per_cw = (te + td) / (2048 * threads)
    n = int(min(1 << 20, max(4096, seconds_target / per_cw)))
    te, td = roundtrip(n)
    return {"value": n / (te + td), "unit": "codewords/s", "cores": threads, "kind": kind,
            "sample": f"{n} codewords: encode + 16-error decode round trip, {threads} threads x one handle, {label}",
            "encode_cw_per_s": n / te, "decode_cw_per_s": n / td}


def host_pipeline(rs, cw_dev, pos8, mag8, stream, reps=3):
    """PCIe-inclusive rates of the host-memory batch API (poporon_encode_batch /
    poporon_decode_batch: pinned 3-slot pipeline, include/poporon_amd.h) on the
    bench's own codewords, copied to host memory.  Reported beside `value`,
    never as it (inputs are not HBM-resident here)."""
    import ctypes as C
    B = cw_dev.shape[0]
    host = cw_dev.cpu().numpy()  # clean codewords (B, 255)
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
    bad = cw_dev.clone()
    P.channel_xor_device(pos8.data_ptr(), mag8.data_ptr(), 16, bad.data_ptr(), N, B, stream)
    torch.cuda.synchronize()
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
    return {"encode_cw_per_s": round(B / e, 1), "encode_GB_per_s_pcie": round(B * (K + NR) / e / 1e9, 2),
            "decode_cw_per_s": round(B / d, 1), "decode_GB_per_s_pcie": round(B * (2 * N + 2) / d / 1e9, 2),
            "codewords": B, "note": "host-memory batch API, PCIe-inclusive (best of %d); not `value`" % reps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-erasure", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory (PCIe) pipeline rates")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes from a rocprofv3 --pmc pass (tools/pmc_traffic.py)")
    args = ap.parse_args()

    world, rank, local = dist_setup()
    dev = torch.device("cuda", local)
    B = args.batch
    first = rank * B  # global codeword index of this rank's shard

    rs = P.Poporon.default(device=local)
    rs.reserve(B)
    stream = torch.cuda.current_stream().cuda_stream

    # synthetic codewords: messages from the counter hash, parity by our encoder
    cw = torch.zeros((B, N), dtype=torch.uint8, device=dev)
    cw[:, :K] = synth_bytes(SEED, first, B, K, dev)
    pos, mag = synth_errors(SEED + 1, first, B, 16, N, dev)
    pos8, mag8 = pos.to(torch.uint8).contiguous(), mag.to(torch.uint8).contiguous()
    okb = torch.zeros(B, dtype=torch.uint8, device=dev)
    corb = torch.zeros(B, dtype=torch.uint8, device=dev)
    base = cw.data_ptr()

    # Every step: encode the batch (parity recomputed in place) and decode one
    # batch of corrupted codewords.  The corruption (the test channel) is not
    # part of the codec: each step decodes its own copy, corrupted before the
    # timed region, so the timed loop holds exactly encode + decode@16 errors.
    # (If the copies do not fit, the channel runs inside the step, in place.)
    rs.encode_batch_device(base, N, base + K, N, K, B, stream)
    torch.cuda.synchronize()
    clean = cw.clone()
    ncopy = args.warmup + args.steps
    copies = ncopy * B * N <= 0.5 * torch.cuda.mem_get_info(dev)[0]
    if copies:
        bad = torch.empty((ncopy, B, N), dtype=torch.uint8, device=dev)
        for k in range(ncopy):
            bad[k].copy_(clean)
            P.channel_xor_device(pos8.data_ptr(), mag8.data_ptr(), 16, bad[k].data_ptr(), N, B, stream)
        torch.cuda.synchronize()

    def step(k):
        rs.encode_batch_device(base, N, base + K, N, K, B, stream)
        if copies:
            d = bad[k].data_ptr()
        else:
            P.channel_xor_device(pos8.data_ptr(), mag8.data_ptr(), 16, base, N, B, stream)
            d = base
        rs.decode_batch_device(d, N, d + K, N, K, B, okb.data_ptr(), corb.data_ptr(), stream=stream)

    for k in range(args.warmup):
        step(k)
    barrier(world)
    rs.timing(True)
    barrier(world)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    barrier(world)
    t1 = time.perf_counter()
    elapsed = allreduce(t1 - t0, dist.ReduceOp.MAX if world > 1 else None, world)
    kt = {k: rs.timing_read(k) for k in (P.KERNEL_ENCODE, P.KERNEL_REMAINDER, P.KERNEL_CORRECT)}
    rs.timing(False)
    dec_out = bad[args.warmup:] if copies else cw[None]

    # verification of the last step (all ranks): every codeword corrected back
    nbad = int((okb != 1).sum()) + int((corb != 16).sum()) + int((cw != clean).any(dim=1).sum())
    nbad += sum(int((dec_out[k] != clean).any(dim=1).sum()) for k in range(dec_out.shape[0]))
    nbad = int(allreduce(nbad, dist.ReduceOp.SUM if world > 1 else None, world))
    if copies:
        del bad, dec_out

    # the same round trip with the channel inside the step, in place (the
    # round-1 bench shape; reported beside value for continuity)
    def step_inplace():
        rs.encode_batch_device(base, N, base + K, N, K, B, stream)
        P.channel_xor_device(pos8.data_ptr(), mag8.data_ptr(), 16, base, N, B, stream)
        rs.decode_batch_device(base, N, base + K, N, K, B, okb.data_ptr(), corb.data_ptr(), stream=stream)
    step_inplace()
    barrier(world)
    tc0 = time.perf_counter()
    for _ in range(args.steps):
        step_inplace()
    barrier(world)
    tch = allreduce(time.perf_counter() - tc0, dist.ReduceOp.MAX if world > 1 else None, world)
    nbad += int(allreduce(int((cw != clean).any(dim=1).sum()) + int((okb != 1).sum()),
                          dist.ReduceOp.SUM if world > 1 else None, world))
    parity_sum = allreduce(float(cw[:, K:].to(torch.int64).sum()), dist.ReduceOp.SUM if world > 1 else None, world)

    total = B * world * args.steps
    value = total / elapsed
    ms_step = elapsed / args.steps * 1e3
    per_kernel = {}
    for k, (ms, n) in kt.items():
        avg = ms / max(1, n)
        per_kernel[P.KERNEL_NAMES[k]] = {"avg_ms": round(avg, 4), "launches": n,
                                         "cw_per_s_per_gpu": round(B / (avg * 1e-3), 1) if avg > 0 else None,
                                         "GB_s_algorithmic": round(B * CW_BYTES / (avg * 1e-3) / 1e9, 1)
                                         if avg > 0 else None}
    enc_ms = kt[P.KERNEL_ENCODE][0] / max(1, kt[P.KERNEL_ENCODE][1])
    dec_ms = (kt[P.KERNEL_REMAINDER][0] / max(1, kt[P.KERNEL_REMAINDER][1]) +
              kt[P.KERNEL_CORRECT][0] / max(1, kt[P.KERNEL_CORRECT][1]))
    dom = max(kt, key=lambda k: kt[k][0])
    dom_avg_s = kt[dom][0] / max(1, kt[dom][1]) * 1e-3
    achieved = B * CW_BYTES / dom_avg_s / 1e9
    traffic = None
    try:
        with open(args.traffic) as f:
            tj = json.load(f)
        traffic = tj.get("kernels", {}).get(P.KERNEL_NAMES[dom], {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    # erasure decode (configs[3]): 32 sorted erasures per codeword, in [0,223)
    erasure = None
    if not args.no_erasure:
        epos, emag = synth_errors(SEED + 2, first, B, 32, K, dev)
        epos, order = epos.sort(dim=1)
        slots = epos.to(torch.uint8).contiguous()
        emag8 = emag.gather(1, order).to(torch.uint8).contiguous()
        cnts = torch.full((B,), 32, dtype=torch.uint8, device=dev)
        rs.encode_batch_device(base, N, base + K, N, K, B, stream)
        eclean = cw.clone()
        es = max(3, args.steps // 2)
        ecopies = (es + 1) * B * N <= 0.5 * torch.cuda.mem_get_info(dev)[0]
        if ecopies:
            ebad = torch.empty((es + 1, B, N), dtype=torch.uint8, device=dev)
            for k in range(es + 1):
                ebad[k].copy_(eclean)
                P.channel_xor_device(slots.data_ptr(), emag8.data_ptr(), 32, ebad[k].data_ptr(), N, B, stream)

        def estep(k):
            if ecopies:
                d = ebad[k].data_ptr()
            else:
                P.channel_xor_device(slots.data_ptr(), emag8.data_ptr(), 32, base, N, B, stream)
                d = base
            rs.decode_batch_device(d, N, d + K, N, K, B, okb.data_ptr(), corb.data_ptr(),
                                   d_positions=slots.data_ptr(), positions_stride=32, d_counts=cnts.data_ptr(),
                                   stream=stream)
        estep(0)
        barrier(world)
        rs.timing(True)
        t2 = time.perf_counter()
        for k in range(es):
            estep(1 + k)
        barrier(world)
        et = allreduce(time.perf_counter() - t2, dist.ReduceOp.MAX if world > 1 else None, world)
        ec = rs.timing_read(P.KERNEL_CORRECT)
        er = rs.timing_read(P.KERNEL_REMAINDER)
        rs.timing(False)
        eout = ebad[1:] if ecopies else cw[None]
        enbad = int((okb != 1).sum()) + sum(int((eout[k] != eclean).any(dim=1).sum()) for k in range(eout.shape[0]))
        enbad = int(allreduce(enbad, dist.ReduceOp.SUM if world > 1 else None, world))
        if ecopies:
            del ebad, eout
        erasure = {"cw_per_s": round(B * world * es / et, 1),
                   "kernel_cw_per_s_per_gpu": round(B / ((ec[0] / ec[1] + er[0] / er[1]) * 1e-3), 1),
                   "verified": enbad == 0,
                   "channel": "outside the timed decodes (one corrupted copy per decode)" if ecopies
                   else "in place, inside the timed decodes"}

    hostp = None
    if world == 1 and not args.no_host:
        hostp = host_pipeline(rs, clean, pos8, mag8, stream)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-hash messages, 16 random-magnitude errors at unique positions per codeword)",
            "config": {"workload": "RS(255,223) round trip: encode + decode with 16 errors per codeword, "
                                   f"{B} codewords per GPU (BASELINE configs[1]+[2]; configs[4] at N=8 is 8x{B})",
                       "codewords_per_gpu": B, "layout": "255-byte codeword rows, stride 255",
                       "code": "poporon_config_rs_default (8, 0x11D, fcr 1, prim 1, 32 roots)"},
            "GB_per_s": round(value * CW_BYTES / 1e9, 2),
            "step": f"encode {B} messages + decode {B} corrupted codewords (16 errors each); the test channel "
                    "corrupts one copy per step before the timed loop" if copies else
                    "encode + channel (in place) + decode",
            "roundtrip_with_channel_cw_per_s": round(B * world * args.steps / tch, 1),
            "hbm_frac_of_peak": round(value * CW_BYTES / 1e9 / (HBM_PEAK_GBS * world), 4),
            "encode_cw_per_s_per_gpu": round(B / (enc_ms * 1e-3), 1),
            "decode_cw_per_s_per_gpu": round(B / (dec_ms * 1e-3), 1),
            "kernels": per_kernel,
            "roofline": {"kernel": P.KERNEL_NAMES[dom], "bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "note": "achieved = 255 B x codewords per launch / average launch time (HIP events, "
                                 "launch stream); the kernel is VALU/LDS-bound, see DESIGN.md"},
            "erasure_decode_32": erasure,
            "host_pipeline": hostp,
            "verified": nbad == 0,
            "parity_checksum": int(parity_sum),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
