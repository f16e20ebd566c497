#!/usr/bin/env python3
"""Device-batch latency by batch size (diagnostic): encode and 16-error decode
of n resident codewords through the C ABI, wall time per call (median of
reps, stream-synchronised), for n from 1 to 2^20.

    python tools/batch_latency.py [--reps 20]

POPORON_AMD_DECODE_PATH=split|single|wave selects the decode route as in the
tests (default: split from 8,192 codewords on)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import devdata  # noqa: E402
import libpoporon_amd as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rs = P.Poporon.default(device=0)
    K, N = 223, 255
    s = torch.cuda.current_stream().cuda_stream
    out = {"path": os.environ.get("POPORON_AMD_DECODE_PATH", "default"), "us": {}}
    for n in (1, 16, 256, 1024, 4096, 8191, 8192, 12288, 16384, 24576, 32768, 65536, 1 << 20):
        cw = torch.zeros((n, N), dtype=torch.uint8, device=dev)
        cw[:, :K] = devdata.synth_bytes(bench.SEED, 0, n, K, dev)
        b = cw.data_ptr()
        rs.encode_batch_device(b, N, b + K, N, K, n, s)
        pos, mag = devdata.synth_errors(bench.SEED + 1, 0, n, 16, N, dev)
        clean = cw.clone()
        bad = clean.clone()
        devdata.channel(pos, mag, 16, bad.data_ptr(), N, n, s)
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        te, td = [], []
        for r in range(a.reps + 2):
            cw.copy_(bad)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), stream=s)
            torch.cuda.synchronize()
            td.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            rs.encode_batch_device(b, N, b + K, N, K, n, s)
            torch.cuda.synchronize()
            te.append(time.perf_counter() - t0)
        assert torch.equal(cw, clean) and int(ok.sum()) == n
        med = lambda v: sorted(v[2:])[len(v[2:]) // 2] * 1e6  # noqa: E731
        out["us"][n] = {"encode": round(med(te), 1), "decode16": round(med(td), 1)}
        print(n, out["us"][n], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
