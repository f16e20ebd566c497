#!/usr/bin/env python3
"""Time the kernels of one or more library builds (experiments).

    python tools/exp_time.py build/a.so build/b.so ...

Each build runs in its own child process (POPORON_AMD_LIB): 2^20 codewords,
encode + channel (16 errors) + decode, 3 warm-up + 10 timed round trips;
prints the average kernel times from the in-library HIP-event timing."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import torch
    import bench
    import libpoporon_amd as P
    import testutil as T
    n, K, N = 1 << 20, 223, 255
    dev = torch.device("cuda", 0)
    rs = P.Poporon.default(device=0)
    rs.reserve(n)
    cw = torch.zeros((n, N), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    T.synth_rows(bench.SEED, 0, n, K, cw.data_ptr(), N, s)
    pos8 = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    mag8 = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    T.synth_errors(bench.SEED + 1, 0, n, 16, N, pos8.data_ptr(), mag8.data_ptr(), False, s)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    cor = torch.zeros(n, dtype=torch.uint8, device=dev)
    b = cw.data_ptr()

    def step():
        rs.encode_batch_device(b, N, b + K, N, K, n, s)
        T.channel_xor(pos8.data_ptr(), mag8.data_ptr(), 16, b, N, n, s)
        rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), stream=s)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / 10 * 1e3
    rs.timing(True)
    for _ in range(10):
        step()
    res = {"step_ms": round(step_ms, 4)}
    for k in P.KERNEL_NAMES:
        ms, c = rs.timing_read(k)
        if c:
            res[P.KERNEL_NAMES[k]] = round(ms / c, 4)
    res["ok"] = int(ok.sum()) == n and bool((cor == 16).all())
    rs.timing(False)
    # erasure decode (32 sorted erasures in the data, configs[3])
    slots = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    emag8 = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    T.synth_errors(bench.SEED + 2, 0, n, 32, K, slots.data_ptr(), emag8.data_ptr(), True, s)
    cnts = torch.full((n,), 32, dtype=torch.uint8, device=dev)
    rs.encode_batch_device(b, N, b + K, N, K, n, s)

    def estep():
        T.channel_xor(slots.data_ptr(), emag8.data_ptr(), 32, b, N, n, s)
        rs.decode_batch_device(b, N, b + K, N, K, n, ok.data_ptr(), cor.data_ptr(), d_positions=slots.data_ptr(),
                               positions_stride=32, d_counts=cnts.data_ptr(), stream=s)
    estep()
    torch.cuda.synchronize()
    rs.timing(True)
    for _ in range(5):
        estep()
    res["erasure_kernels_ms"] = round(sum(ms / c for ms, c in (rs.timing_read(k) for k in P.KERNEL_NAMES) if c), 4)
    for k in P.KERNEL_NAMES:
        ms, c = rs.timing_read(k)
        if c and "erasure" in P.KERNEL_NAMES[k]:
            res["era_k_ms"] = round(ms / c, 4)
    res["erasure_ok"] = int(ok.sum()) == n
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1:] == ["--child"]:
        child()
        sys.exit(0)
    for lib in sys.argv[1:]:
        env = dict(os.environ, POPORON_AMD_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=300)
        out = r.stdout.strip().splitlines()
        print(f"{os.path.basename(lib)}: {out[-1] if out else 'FAILED ' + r.stderr[-300:]}", flush=True)
