#!/usr/bin/env python3
"""Batch calls issued right after a single call (diagnostic):
a 2^20-codeword device encode and 16-error decode on a handle whose
single-call server (rs_serve_k) a poporon_encode has just left resident,
against the same calls with no single call before them.  Wall time per call
(stream-synchronised), median of reps; the results must be identical.

    python tools/server_batch.py [--reps 15]

POPORON_AMD_LIB selects the build (tools/variants.sh), POPORON_AMD_SERVE=0
turns the server off."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import devdata  # noqa: E402
import libpoporon_amd as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rs = P.Poporon.default(device=0)
    K, N, n = 223, 255, 1 << 20
    s = torch.cuda.current_stream().cuda_stream
    cw = torch.zeros((n, N), dtype=torch.uint8, device=dev)
    cw[:, :K] = devdata.synth_bytes(bench.SEED, 0, n, K, dev)
    b = cw.data_ptr()
    rs.encode_batch_device(b, N, b + K, N, K, n, s)
    pos, mag = devdata.synth_errors(bench.SEED + 1, 0, n, 16, N, dev)
    clean = cw.clone()
    bad = clean.clone()
    devdata.channel(pos, mag, 16, bad.data_ptr(), N, n, s)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    msg = np.arange(K, dtype=np.uint8)
    want_single = rs.encode(msg)
    res = {}
    for case in ("alone", "after_single"):
        te, td = [], []
        for r in range(a.reps + 2):
            cw.copy_(bad)
            torch.cuda.synchronize()
            if case == "after_single":
                assert (rs.encode(msg) == want_single).all()
            t0 = time.perf_counter()
            rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), stream=s)
            torch.cuda.synchronize()
            td.append(time.perf_counter() - t0)
            assert torch.equal(cw, clean) and int(ok.sum()) == n
            if case == "after_single":
                assert (rs.encode(msg) == want_single).all()
            t0 = time.perf_counter()
            rs.encode_batch_device(b, N, b + K, N, K, n, s)
            torch.cuda.synchronize()
            te.append(time.perf_counter() - t0)
            assert torch.equal(cw, clean)
        med = lambda v: sorted(v[2:])[len(v[2:]) // 2] * 1e3  # noqa: E731
        res[case] = {"encode_ms": round(med(te), 4), "decode16_ms": round(med(td), 4),
                     "encode_max_ms": round(max(te[2:]) * 1e3, 4), "decode16_max_ms": round(max(td[2:]) * 1e3, 4)}
        print(case, res[case], flush=True)
    res["lib"] = os.path.basename(P.LIB_PATH)
    res["serve"] = os.environ.get("POPORON_AMD_SERVE", "1")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
