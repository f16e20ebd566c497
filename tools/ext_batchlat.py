#!/usr/bin/env python3
"""Wall time per external-syndrome device decode call
(poporon_decode_batch_syndrome_device) over batch sizes: rs_wave_k (one
codeword per wave, POPORON_AMD_DECODE_PATH=wave; the general kernel for
codes with fewer roots, =single) against the split kernels fed by
rsk_ext_syn (=split), on rows with up to t errors and their own syndromes.

    python tools/ext_batchlat.py [--params 8,0x11D,1,1,32] [--reps 10]"""
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
    ap.add_argument("--params", default="8,0x11D,1,1,32")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    params = tuple(int(x, 0) for x in a.params.split(","))
    nr = params[4]
    k = 255 - nr
    t = nr // 2
    handles = {}
    for path in ("one_kernel", "split"):
        os.environ["POPORON_AMD_DECODE_PATH"] = "split" if path == "split" else ("wave" if nr == 32 else "single")
        handles[path] = P.Poporon(*params)
    os.environ.pop("POPORON_AMD_DECODE_PATH")
    h = handles["split"]
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(1)
    nmax = 1 << 18
    data = rng.integers(0, 256, (nmax, k), dtype=np.uint8)
    clean = np.concatenate([data, h.encode_batch(data)], 1)
    bad = clean.copy()
    for c in range(nmax):
        pos = rng.permutation(255)[:t]
        bad[c, pos] ^= rng.integers(1, 256, t, dtype=np.uint8)
    src = torch.from_numpy(bad).cuda()
    syn = torch.zeros((nmax, nr), dtype=torch.int16, device="cuda")
    nz = torch.zeros(nmax, dtype=torch.uint8, device="cuda")
    b = src.data_ptr()
    h.syndrome_batch_device(b, 255, b + k, 255, k, nmax, syn.data_ptr(), nr, nz.data_ptr(), s)
    torch.cuda.synchronize()
    ref = torch.from_numpy(clean).cuda()
    res = {}
    for n in (4096, 16384, 65536, 262144):
        row = {}
        for path, hh in handles.items():
            buf = src[:n].clone()
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            bb = buf.data_ptr()
            ts = []
            for r in range(a.reps + 1):
                buf.copy_(src[:n])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hh.decode_batch_syndrome_device(bb, 255, bb + k, 255, k, n, syn.data_ptr(), nr, ok.data_ptr(), 0, s)
                torch.cuda.synchronize()
                if r:
                    ts.append(time.perf_counter() - t0)
            assert bool((ok == 1).all()) and bool((buf == ref[:n]).all()), (path, n)
            row[path + "_us"] = round(float(np.median(ts)) * 1e6, 1)
        res[n] = row
        print(n, json.dumps(row), flush=True)
    print(json.dumps({"params": a.params, "per_call_us": res}))


if __name__ == "__main__":
    main()
