"""Multi-process (gloo, world size 2) checks of the N>1 bookkeeping of bench.py.

The GPU path shards codewords by contiguous global ranges with no data-path
collective; here, on CPU: every rank generates its shard from the global
index (counter hash) and the concatenation equals the single-process data;
errors likewise; max-time and sum reductions behave as bench.py uses them.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import libpoporon_amd as P


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = P.shard_range(total, rank, world)
    data = bench.synth_bytes(bench.SEED, lo, hi - lo, 223, "cpu")
    pos, mag = bench.synth_errors(bench.SEED + 1, lo, hi - lo, 16, 255, "cpu")
    t = bench.allreduce(float(rank + 1), dist.ReduceOp.MAX, world, device="cpu")
    s = bench.allreduce(float(hi - lo), dist.ReduceOp.SUM, world, device="cpu")
    q.put((rank, data.numpy().copy(), pos.numpy().copy(), mag.numpy().copy(), t, s))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [1000, 1 << 12])
def test_two_rank_sharding_matches_single(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = bench.synth_bytes(bench.SEED, 0, total, 223, "cpu").numpy()
    fpos, fmag = bench.synth_errors(bench.SEED + 1, 0, total, 16, 255, "cpu")
    import numpy as np
    assert (np.concatenate([r[1] for r in res]) == full).all()
    assert (np.concatenate([r[2] for r in res]) == fpos.numpy()).all()
    assert (np.concatenate([r[3] for r in res]) == fmag.numpy()).all()
    assert all(r[4] == 2.0 for r in res)          # max over ranks
    assert all(r[5] == float(total) for r in res)  # sum of shard sizes


def test_error_positions_unique_and_in_range():
    pos, mag = bench.synth_errors(bench.SEED + 1, 123, 512, 16, 255, "cpu")
    assert int(pos.min()) >= 0 and int(pos.max()) < 255
    assert all(len(set(row.tolist())) == 16 for row in pos)
    assert int(mag.min()) >= 1
    epos, _ = bench.synth_errors(bench.SEED + 2, 0, 256, 32, 223, "cpu")
    assert int(epos.max()) < 223 and all(len(set(r.tolist())) == 32 for r in epos)
