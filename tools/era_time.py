#!/usr/bin/env python3
"""Per-kernel times of the erasure decode (configs[3]: 2^20 codewords, 32
sorted erasures each), from the library's HIP-event kernel timers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import devdata  # noqa: E402
import libpoporon_amd as P  # noqa: E402


def main():
    n, K, N = 1 << 20, 223, 255
    dev = torch.device("cuda", 0)
    cw = torch.zeros((n, N), dtype=torch.uint8, device=dev)
    cw[:, :K] = devdata.synth_bytes(bench.SEED, 0, n, K, dev)
    pos, mag = devdata.synth_errors(bench.SEED + 2, 0, n, 32, K, dev)
    pos = pos.sort(dim=1).values
    pl = pos.long()
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    cor = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    rs = P.Poporon.default(device=0)
    b = cw.data_ptr()
    rs.encode_batch_device(b, N, b + K, N, K, n, s)
    clean = cw.clone()
    slots = pos.to(torch.uint8).contiguous()
    cnt = torch.full((n,), 32, dtype=torch.uint8, device=dev)
    acc = {}
    for rep in range(8):
        cw.copy_(clean)
        cw.scatter_(1, pl, cw.gather(1, pl) ^ mag)
        torch.cuda.synchronize()
        rs.timing(True)
        rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), d_positions=slots.data_ptr(),
                               positions_stride=32, d_counts=cnt.data_ptr(), stream=s)
        torch.cuda.synchronize()
        for k in P.KERNEL_NAMES:
            ms, c = rs.timing_read(k)
            if c and rep:
                acc.setdefault(k, []).append(ms)
        rs.timing(False)
        assert torch.equal(cw, clean) and int(ok.sum()) == n
    for k, v in acc.items():
        print(f"{P.KERNEL_NAMES[k] if isinstance(P.KERNEL_NAMES, dict) else k}: {sum(v) / len(v):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
