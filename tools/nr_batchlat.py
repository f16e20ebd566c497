#!/usr/bin/env python3
"""Wall time per errors-only device decode call of a byte-symbol code with
fewer than 32 roots, general kernel (rs_generic.hip) against the split
kernels (POPORON_AMD_DECODE_PATH=split, npar = nr), over batch sizes: where
the split path starts to pay (api.cpp launch_decode, h->nrsplit).

    python tools/nr_batchlat.py [--params 8,0x11D,1,1,16] [--reps 20]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="8,0x11D,1,1,16")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    params = tuple(int(x, 0) for x in a.params.split(","))
    nr = params[4]
    k = 255 - nr
    t = nr // 2
    handles = {}
    for path in ("general", "split"):
        os.environ["POPORON_AMD_DECODE_PATH"] = "split" if path == "split" else "single"
        handles[path] = P.Poporon(*params)
    os.environ.pop("POPORON_AMD_DECODE_PATH")
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(1)
    nmax = 1 << 16
    data = rng.integers(0, 256, (nmax, k), dtype=np.uint8)
    clean = np.concatenate([data, handles["split"].encode_batch(data)], 1)
    bad = clean.copy()
    for c in range(nmax):
        pos = rng.permutation(255)[:t]
        bad[c, pos] ^= rng.integers(1, 256, t, dtype=np.uint8)
    src = torch.from_numpy(bad).cuda()
    res = {}
    for n in (1024, 2048, 4096, 8192, 12288, 16384, 32768, 65536):
        row = {}
        for path, h in handles.items():
            buf = src[:n].clone()
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            b = buf.data_ptr()
            ts = []
            for r in range(a.reps + 1):
                buf.copy_(src[:n])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                h.decode_batch_device(b, 255, b + k, 255, k, n, ok.data_ptr(), stream=s)
                torch.cuda.synchronize()
                if r:
                    ts.append(time.perf_counter() - t0)
            assert bool((ok == 1).all()) and (buf.cpu().numpy() == clean[:n]).all(), (path, n)
            row[path + "_us"] = round(float(np.median(ts)) * 1e6, 1)
        res[n] = row
        print(n, json.dumps(row), flush=True)
    print(json.dumps({"params": a.params, "per_call_us": res}))


if __name__ == "__main__":
    main()
