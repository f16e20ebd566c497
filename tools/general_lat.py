#!/usr/bin/env python3
"""Latency and throughput of every parameter set of the reference's own
tests (tests/golden/rs_params_golden.npz): single calls (poporon_encode /
poporon_decode through ctypes, t errors) and device batches of 64, 4,096 and
65,536 codewords (t errors each), with the reference's own single calls
(oracle/_ref, the same ctypes path, one host core) beside them.

    python tools/general_lat.py [--calls 100]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libpoporon_amd as P  # noqa: E402


def _errors(rng, cw, nn, nerr):
    for c in range(len(cw)):
        pos = rng.permutation(cw.shape[1])[:nerr]
        cw[c, pos] ^= rng.integers(1, nn + 1, nerr).astype(np.uint8)
    return cw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=100)
    ap.add_argument("--path", default="", help="POPORON_AMD_GENERIC: wave | lane (default: by batch size)")
    a = ap.parse_args()
    if a.path:
        os.environ["POPORON_AMD_GENERIC"] = a.path
    params = np.load(os.path.join(ROOT, "tests", "golden", "rs_params_golden.npz"))["params"]
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for prm in params:
        m, poly, fcr, prim, nr = (int(x) for x in prm)
        nn = (1 << m) - 1
        k = nn - nr
        t = nr // 2
        h = P.Poporon(m, poly, fcr, prim, nr)
        rng = np.random.default_rng(nr + m)
        msgs = rng.integers(0, nn + 1, (a.calls, k), dtype=np.uint8)
        h.encode(msgs[0])
        t0 = time.perf_counter()
        pars = [h.encode(x) for x in msgs]
        te = (time.perf_counter() - t0) / a.calls
        clean = np.concatenate([msgs, np.array(pars)], 1)
        bad = _errors(rng, clean.copy(), nn, t)
        h.decode(bad[0, :k], bad[0, k:])
        t0 = time.perf_counter()
        res = [h.decode(cw[:k], cw[k:]) for cw in bad]
        td = (time.perf_counter() - t0) / a.calls
        okfrac = float(np.mean([r[0] for r in res]))  # 0 for two sets: the reference's own failures (oracle)
        row = {"encode_us": round(te * 1e6, 1), "decode_us": round(td * 1e6, 1), "single_ok": okfrac}
        # the reference itself (oracle/_ref, compiled from /root/reference/src), same calls through ctypes
        from oracle import Reference, reference_available
        if reference_available():
            ref = Reference(m, poly, fcr, prim, nr)
            t0 = time.perf_counter()
            for x in msgs:
                ref.encode(x)
            row["ref_encode_us"] = round((time.perf_counter() - t0) / a.calls * 1e6, 1)
            t0 = time.perf_counter()
            for cw in bad:
                ref.decode(cw[:k], cw[k:])
            row["ref_decode_us"] = round((time.perf_counter() - t0) / a.calls * 1e6, 1)
            ref.close()
        for n in (64, 4096, 65536):
            data = rng.integers(0, nn + 1, (n, k), dtype=np.uint8)
            cw = np.concatenate([data, h.encode_batch(data)], 1)
            src = torch.from_numpy(_errors(rng, cw.copy(), nn, t)).cuda()
            ref = torch.from_numpy(cw).cuda()
            buf = src.clone()
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            b = buf.data_ptr()
            ts = []
            for r in range(6):
                buf.copy_(src)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                h.decode_batch_device(b, nn, b + k, nn, k, n, ok.data_ptr(), stream=s)
                torch.cuda.synchronize()
                if r:
                    ts.append(time.perf_counter() - t0)
            if okfrac == 1.0:
                assert bool((ok == 1).all()) and bool((buf == ref).all()), (prm, n)
            row[f"batch{n}_us"] = round(float(np.median(ts)) * 1e6, 1)
            # device encode of the same rows (parity into a separate buffer)
            dd = torch.from_numpy(np.ascontiguousarray(data)).cuda()
            pp = torch.zeros((n, nr), dtype=torch.uint8, device="cuda")
            ts = []
            for r in range(6):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                h.encode_batch_device(dd.data_ptr(), k, pp.data_ptr(), nr, k, n, stream=s)
                torch.cuda.synchronize()
                if r:
                    ts.append(time.perf_counter() - t0)
            assert bool((pp == ref[:, k:]).all()), (prm, n, "encode")
            row[f"enc{n}_us"] = round(float(np.median(ts)) * 1e6, 1)
        name = f"m{m} {hex(poly)} fcr{fcr} prim{prim} nr{nr}"
        out[name] = row
        print(name, json.dumps(row), flush=True)
        h.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
