"""Multi-process (gloo) tests of bench.py's multi-rank path, on CPU.

`bench.py --gpus N` starts N ranks itself (torch.distributed.run as a child
process, before any GPU use).  Here the same launcher, the configs[4] strong
split (libpoporon_amd's partition), the weak-scaling shard offsets and the
rank reductions run with tests/bench_cpu_backend.py, which replaces the HIP
codec by the CPU oracle.  The configs[4] checksum must be identical for every
rank count, and n_gpus must equal --gpus.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
import libpoporon_amd as P
import testutil as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(gpus, extra=(), env_extra=None):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "tests.bench_cpu_backend",
           "--batch", "256", "--steps", "1", "--warmup", "0", "--c4-total", "1000", "--c4-chunk", "300",
           "--c4-reps", "1", *extra]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_launcher_ranks_and_checksum():
    one = _line(_run(1))
    two = _line(_run(2))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["verified"] and two["verified"]
    # configs[4]: the same 1000 codewords however they are split
    assert one["configs4"]["codewords_per_gpu"] == 1000 and two["configs4"]["codewords_per_gpu"] == 500
    assert one["parity_checksum"] == two["parity_checksum"] == one["configs4"]["parity_checksum"]
    # each rank's share of the checksum, over its own contiguous range
    rc = two["configs4"]["rank_checksums"]
    assert [r["range"] for r in rc] == [[0, 500], [500, 1000]]
    assert sum(r["out"] for r in rc) % (1 << 64) == two["parity_checksum"]
    assert all(r["in"] == r["out"] for r in rc)  # every rank's range decoded back to its encoded rows
    from oracle import Oracle
    msgs = T.synth_rows_cpu(bench.SEED + 4, 0, 1000, 223)
    cw = np.concatenate([msgs, Oracle().encode_batch(msgs)], 1)
    assert T.checksum_cpu(cw, 0) == one["parity_checksum"]
    # weak scaling: rank r owns rows [r*B, (r+1)*B), the line counts both ranks
    assert two["config"]["codewords_per_gpu"] == 256
    msgs2 = T.synth_rows_cpu(bench.SEED, 0, 512, 223)
    cw2 = np.concatenate([msgs2, Oracle().encode_batch(msgs2)], 1)
    assert T.checksum_cpu(cw2, 0) == two["weak_checksum"]


def test_gpus_must_match_world_size():
    r = _run(1, env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


@pytest.mark.parametrize("total,world", [(1000, 2), (4096, 3), (1 << 20, 8), (7, 8)])
def test_partition_matches_library(total, world):
    """bench.shard is the library's partition (poporon_amd_multi_range)."""
    got = [bench.shard(total, r, world) for r in range(world)]
    assert got == [P.shard_range(total, r, world) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == total
    assert all(got[i][1] == got[i + 1][0] for i in range(world - 1))


def test_shards_reproduce_single_process_rows():
    """Rows, errors and checksums depend only on the global row index."""
    total, world = 1000, 3
    full = T.synth_rows_cpu(bench.SEED, 0, total, 223)
    fpos, fmag = T.synth_errors_cpu(bench.SEED + 1, 0, total, 16, 255)
    parts = [bench.shard(total, r, world) for r in range(world)]
    assert (np.concatenate([T.synth_rows_cpu(bench.SEED, a, b - a, 223) for a, b in parts]) == full).all()
    ep = [T.synth_errors_cpu(bench.SEED + 1, a, b - a, 16, 255) for a, b in parts]
    assert (np.concatenate([e[0] for e in ep]) == fpos).all() and (np.concatenate([e[1] for e in ep]) == fmag).all()
    cs = sum(T.checksum_cpu(full[a:b], a) for a, b in parts) & ((1 << 64) - 1)
    assert cs == T.checksum_cpu(full, 0)


def test_error_patterns_unique_and_in_range():
    pos, mag = T.synth_errors_cpu(bench.SEED + 1, 123, 512, 16, 255)
    assert int(pos.min()) >= 0 and int(pos.max()) < 255
    assert all(len(set(row.tolist())) == 16 for row in pos)
    assert int(mag.min()) >= 1
    epos, emag = T.synth_errors_cpu(bench.SEED + 2, 0, 256, 32, 223, sorted_positions=True)
    assert int(epos.max()) < 223 and all(len(set(r.tolist())) == 32 for r in epos)
    assert (np.diff(epos.astype(np.int32), axis=1) > 0).all()
    # sorting keeps each magnitude with its position
    up, um = T.synth_errors_cpu(bench.SEED + 2, 0, 256, 32, 223)
    for r in range(256):
        assert dict(zip(up[r].tolist(), um[r].tolist())) == dict(zip(epos[r].tolist(), emag[r].tolist()))


def test_scatter_from_rank0():
    """--c4-scatter: rank 0 sends each rank its range point-to-point (gloo
    here, RCCL send/recv on GPUs); every codeword decodes, and the checksum
    equals the encoded batch's, computed independently here."""
    r = _line(_run(2, ("--no-c4", "--c4-scatter", "600", "--c4-reps", "1")))
    sc = r["configs4_scatter"]
    assert r["verified"] and sc["verified"] and sc["n_gpus"] == 2 and sc["total_codewords"] == 600
    assert sc["scatter_ms"] > 0 and sc["scatter_decode_ms"] >= sc["scatter_ms"]
    from oracle import Oracle
    msgs = T.synth_rows_cpu(bench.SEED + 11, 0, 600, 223)
    cw = np.concatenate([msgs, Oracle().encode_batch(msgs)], 1)
    assert T.checksum_cpu(cw, 0) == sc["parity_checksum"]
    one = _line(_run(1, ("--no-c4", "--c4-scatter", "600")))
    assert "configs4_scatter" not in one  # nothing to move on one rank
