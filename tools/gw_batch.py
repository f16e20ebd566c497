#!/usr/bin/env python3
"""Device batch decodes of one general parameter set, for rocprofv3 (kernel
trace or --pmc passes): `reps` decodes of n codewords with t errors each on
the default routing (POPORON_AMD_GENERIC=wave|lane to force a family).

    python tools/gw_batch.py [--params 8,0x11d,1,1,100] [--n 65536] [--reps 5]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libpoporon_amd as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="8,0x11d,1,1,100")
    ap.add_argument("--n", type=int, default=1 << 16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-check", action="store_true", help="experiment builds (GW_PHASE_STOP): skip the result check")
    a = ap.parse_args()
    m, poly, fcr, prim, nr = (int(x, 0) for x in a.params.split(","))
    nn = (1 << m) - 1
    k, t = nn - nr, nr // 2
    h = P.Poporon(m, poly, fcr, prim, nr)
    rng = np.random.default_rng(5)
    data = rng.integers(0, nn + 1, (a.n, k), dtype=np.uint8)
    cw = np.concatenate([data, h.encode_batch(data)], 1)
    pos = np.argsort(rng.random((a.n, nn)), axis=1)[:, :t]
    np.bitwise_xor.at(cw, (np.arange(a.n)[:, None], pos), rng.integers(1, nn + 1, (a.n, t), dtype=np.uint8))
    src = torch.from_numpy(cw).cuda()
    buf = src.clone()
    ok = torch.zeros(a.n, dtype=torch.uint8, device="cuda")
    cor = torch.zeros(a.n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    b = buf.data_ptr()
    ts = []
    for _ in range(a.reps):
        buf.copy_(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.decode_batch_device(b, nn, b + k, nn, k, a.n, ok.data_ptr(), cor.data_ptr(), stream=s)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    if not a.no_check:
        assert bool((ok == 1).all()) and bool((cor == t).all()), "decode failed"
    print(f"RS({nn},{k}) n={a.n}: {1e3 * min(ts):.3f} ms best, {a.n / min(ts) / 1e6:.1f} M cw/s")


if __name__ == "__main__":
    main()
