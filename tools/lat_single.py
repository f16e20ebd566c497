#!/usr/bin/env python3
"""Single-call latency (the reference's calling pattern): bench.call_latency
on its own, plus a rocprofv3-friendly loop.  python tools/lat_single.py [calls]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    import torch
    torch.cuda.set_device(0)
    be = bench.GpuBackend(0)
    for _ in range(2):
        r = bench.call_latency(be, calls)
    print(json.dumps(r))


if __name__ == "__main__":
    main()
