#!/usr/bin/env python3
"""Stage ablation driver for PMC collection: one correction-kernel dispatch per
stop_at value (1, 2, 3, 4, 0), in that order, each preceded by a warm-up
dispatch of the same setting.  Run under rocprofv3 --pmc ...; the per-dispatch
counter rows then map to stages by dispatch order (tools/pmc_stages.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench
import devdata  # noqa: E402
import libpoporon_amd as P  # noqa: E402

STOPS = (1, 2, 3, 4, 0)


def main():
    n, K, N = 1 << 20, 223, 255
    dev = torch.device("cuda", 0)
    cw0 = torch.zeros((n, N), dtype=torch.uint8, device=dev)
    cw0[:, :K] = devdata.synth_bytes(bench.SEED, 0, n, K, dev)
    pos, mag = devdata.synth_errors(bench.SEED + 1, 0, n, 16, N, dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    cor = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for stop in STOPS:
        os.environ["POPORON_AMD_STOP_AT"] = str(stop)
        rs = P.Poporon.default(device=0)
        cw = cw0.clone()
        b = cw.data_ptr()
        rs.encode_batch_device(b, N, b + K, N, K, n, s)
        clean = cw.clone()
        for _ in range(2):
            cw.copy_(clean)
            cw.scatter_(1, pos, cw.gather(1, pos) ^ mag)
            rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), stream=s)
        torch.cuda.synchronize()
        rs.close()
    print("ablate_pmc done", STOPS)


if __name__ == "__main__":
    main()
