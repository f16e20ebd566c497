#!/usr/bin/env python3
"""Per-kernel times of experiment builds through bench.py (one child per build).

    python tools/exp_bench.py build/a.so build/b.so ...

Runs `bench.py --no-cpu-baseline --no-host --no-c4 --no-latency --steps 6`
with POPORON_AMD_LIB pointing at each build and prints the kernel averages of
the decode16, erasure32 and errata16e8 lines."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

for lib in sys.argv[1:]:
    env = dict(os.environ, POPORON_AMD_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-host", "--no-c4",
                        "--no-latency", "--no-mixed", "--no-general", "--steps", "6"], env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if not line:
        print(os.path.basename(lib), "FAILED", r.stderr[-400:], flush=True)
        continue
    d = json.loads(line[-1])
    out = {"value": d["value"], "verified": d.get("verified"), "encode": d["roofline_modes"]["encode"]["kernels_ms"],
           "decode16": d["roofline_modes"]["decode16"]["kernels_ms"]}
    for k in ("erasure_decode_32", "errata_decode_16e8"):
        out[k] = {"cw_per_s": d[k]["cw_per_s"], "ms": d[k]["kernels_avg_ms"]}
    print(os.path.basename(lib), json.dumps(out), flush=True)
