#!/usr/bin/env python3
"""Same-box A/B of the bit-sliced encoder prototype (tools/probes/bitslice_enc.hip,
built into tools/probes/_build/libbs{0,1,2}.so) against the product's
rs_lfsr_k<ENCODE> (poporon_encode_batch_device), at 2^20 and 2^23 codewords
in the wire layout.  BS_MODE 0's parity must equal the product encoder's
byte for byte (which the GPU tests pin to the reference's golden vectors);
modes 1 / 2 time the LFSR steps alone / the gathers + transposes alone.

    python tools/probes/bitslice_run.py [--reps 5] [--sizes 20,23]"""
import argparse
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libpoporon_amd as P  # noqa: E402
import testutil as T  # noqa: E402

K, N = 223, 255


def timed(fn, reps, s):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sizes", default="20,23")
    a = ap.parse_args()
    libs = {m: C.CDLL(os.path.join(HERE, "_build", f"libbs{m}.so")) for m in (0, 1, 2)}
    for lib in libs.values():
        lib.bs_encode.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    rs = P.Poporon.default()
    st = torch.cuda.current_stream()
    s = st.cuda_stream
    res = {}
    for lg in (int(x) for x in a.sizes.split(",")):
        n = 1 << lg
        rows = torch.empty((n, N), dtype=torch.uint8, device="cuda")
        T.synth_rows(0xB175, 0, n, K, rows.data_ptr(), N, s)
        b = rows.data_ptr()
        rs.encode_batch_device(b, N, b + K, N, K, n, s)
        out = rows.clone()
        out[:, K:] = 0
        sink = torch.zeros(n // 32 + 64, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        libs[0].bs_encode(out.data_ptr(), out.data_ptr(), n, sink.data_ptr(), s)
        torch.cuda.synchronize()
        nbad = int((out[:, K:] != rows[:, K:]).any(dim=1).sum())
        r = {"codewords": n, "rows_with_parity_mismatch": nbad}
        r["product_rs_lfsr_k_ms"] = timed(lambda: rs.encode_batch_device(b, N, b + K, N, K, n, s), a.reps, st)
        for m, name in ((0, "bitsliced_full_ms"), (1, "bitsliced_lfsr_only_ms"), (2, "bitsliced_gather_only_ms")):
            r[name] = timed(lambda: libs[m].bs_encode(out.data_ptr(), out.data_ptr(), n, sink.data_ptr(), s), a.reps,
                            st)
        torch.cuda.synchronize()
        r["rows_with_parity_mismatch_after_timing"] = int((out[:, K:] != rows[:, K:]).any(dim=1).sum())
        r["per_2^20_ms"] = {k: round(v * (1 << 20) / n, 4) for k, v in r.items() if k.endswith("_ms")}
        res[f"2^{lg}"] = r
        print(json.dumps({f"2^{lg}": r}), flush=True)
        del rows, out, sink
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
