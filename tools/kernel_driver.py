#!/usr/bin/env python3
"""Minimal driver for profiling: the bench's workloads through the C ABI and
nothing else (no CPU baseline, no extra passes).  Used under rocprofv3 by
tools/gpu_session.sh (steps prof / pmc / traffic).

    python tools/kernel_driver.py [--n 1048576] [--reps 5] [--mode roundtrip|erasure]

As in bench.py, the encodes rotate over 3 message buffers and every decode
works on its own corrupted copy made before the profiled loop, so no launch
re-reads a buffer the previous launch left in the Infinity Cache.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import devdata  # noqa: E402
import libpoporon_amd as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", default="roundtrip", choices=["roundtrip", "erasure", "errata", "mixed"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rs = P.Poporon.default(device=0)
    rs.reserve(a.n)
    K, N = 223, 255
    cw = torch.zeros((a.n, N), dtype=torch.uint8, device=dev)
    cw[:, :K] = devdata.synth_bytes(bench.SEED, 0, a.n, K, dev)
    ok = torch.zeros(a.n, dtype=torch.uint8, device=dev)
    cor = torch.zeros(a.n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    if a.mode == "roundtrip":
        pos, mag = devdata.synth_errors(bench.SEED + 1, 0, a.n, 16, N, dev)
        kw = {}
        want = 16
    elif a.mode == "erasure":
        pos, mag = devdata.synth_errors(bench.SEED + 2, 0, a.n, 32, K, dev)
        pos = pos.sort(dim=1).values
        slots = pos.to(torch.uint8).contiguous()
        cnt = torch.full((a.n,), 32, dtype=torch.uint8, device=dev)
        kw = dict(d_positions=slots.data_ptr(), positions_stride=32, d_counts=cnt.data_ptr())
        want = 32
    elif a.mode == "mixed":  # bench.py decode_mixed: binomial(255, 0.045) errors per codeword, capped at 24
        pos, mag = devdata.synth_errors(bench.SEED + 10, 0, a.n, bench.MIXED_CAP, N, dev)
        ne = torch.from_numpy(bench.mixed_counts(0, a.n)).to(dev)
        mag = mag * (torch.arange(bench.MIXED_CAP, device=dev)[None, :] < ne[:, None].long()).to(mag.dtype)
        kw = {}
        want = None
    else:  # bench.py errata16e8: 24 sorted positions, every third an error, the rest 16 erasure slots
        pos, mag = devdata.synth_errors(bench.SEED + 9, 0, a.n, 24, K, dev)
        pos = pos.sort(dim=1).values
        slots = torch.zeros((a.n, 32), dtype=torch.uint8, device=dev)
        slots[:, :16] = pos[:, [k for k in range(24) if k % 3 != 2]].to(torch.uint8)
        cnt = torch.full((a.n,), 16, dtype=torch.uint8, device=dev)
        kw = dict(d_positions=slots.data_ptr(), positions_stride=32, d_counts=cnt.data_ptr())
        want = 24
    pos8, mag8 = pos.to(torch.uint8).contiguous(), mag.to(torch.uint8).contiguous()
    b = cw.data_ptr()
    rs.encode_batch_device(b, N, b + K, N, K, a.n, s)
    enc = [cw] + [cw.clone() for _ in range(2)]
    bad = []
    for _ in range(a.reps):
        c = cw.clone()
        devdata.channel(pos8, mag8, pos8.shape[1], c.data_ptr(), N, a.n, s)
        bad.append(c)
    torch.cuda.synchronize()
    for r in range(a.reps):
        e = enc[r % len(enc)].data_ptr()
        rs.encode_batch_device(e, N, e + K, N, K, a.n, s)
        d = bad[r].data_ptr()
        rs.decode_batch_device(d, N, d + K, N, K, a.n, ok.data_ptr(), cor.data_ptr(), stream=s, **kw)
    torch.cuda.synchronize()
    if want is None:  # mixed: the codewords past t fail or miscorrect as the reference does
        print("driver ok", a.mode, a.n, a.reps, "ok", int(ok.sum()))
        return
    assert int(ok.sum()) == a.n and bool((cor == want).all()), "decode failures"
    if a.mode != "errata":  # errata: the reference applies root n's magnitude at slot n (not restored)
        assert all(bool((x == cw).all()) for x in bad + enc), "decoded bytes differ"
    print("driver ok", a.mode, a.n, a.reps)


if __name__ == "__main__":
    main()
