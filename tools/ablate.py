#!/usr/bin/env python3
"""Stage ablation of the correction kernel (profiling aid).

For stop_at = 1..4 the kernel returns after: syndrome load, erasure+BM, Omega,
Chien; 0 = full decode (Forney + apply on top).  Prints the average correction-kernel time (HIP events)
for each, on 2^20 codewords with 16 errors (or 32 erasures with --erasure).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench
import devdata  # noqa: E402
import libpoporon_amd as P  # noqa: E402


def main():
    erasure = "--erasure" in sys.argv
    n, K, N = 1 << 20, 223, 255
    dev = torch.device("cuda", 0)
    cw0 = torch.zeros((n, N), dtype=torch.uint8, device=dev)
    cw0[:, :K] = devdata.synth_bytes(bench.SEED, 0, n, K, dev)
    if erasure:
        pos, mag = devdata.synth_errors(bench.SEED + 2, 0, n, 32, K, dev)
        pos = pos.sort(dim=1).values
    else:
        pos, mag = devdata.synth_errors(bench.SEED + 1, 0, n, 16, N, dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    cor = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for stop in (1, 2, 3, 4, 0):
        os.environ["POPORON_AMD_STOP_AT"] = str(stop)
        rs = P.Poporon.default(device=0)
        cw = cw0.clone()
        b = cw.data_ptr()
        rs.encode_batch_device(b, N, b + K, N, K, n, s)
        clean = cw.clone()
        kw = {}
        if erasure:
            slots = pos.to(torch.uint8).contiguous()
            cnt = torch.full((n,), 32, dtype=torch.uint8, device=dev)
            kw = dict(d_positions=slots.data_ptr(), positions_stride=32, d_counts=cnt.data_ptr())
        times = []
        for rep in range(6):
            cw.copy_(clean)
            pl = pos.long()
            cw.scatter_(1, pl, cw.gather(1, pl) ^ mag)
            torch.cuda.synchronize()
            rs.timing(True)
            rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), stream=s, **kw)
            ms, _ = rs.timing_read(P.KERNEL_CORRECT)
            rs.timing(False)
            if rep:
                times.append(ms)
        print(f"stop_at={stop}: correct kernel {sum(times)/len(times):.4f} ms  ok={int(ok.sum())}", flush=True)
        rs.close()
    os.environ.pop("POPORON_AMD_STOP_AT")


if __name__ == "__main__":
    main()
