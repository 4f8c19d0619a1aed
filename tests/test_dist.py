"""CPU: the N>1 path (one process per GPU) with world_size-2 gloo ranks.

Each rank takes its byte-balanced contiguous shard (zero-packet_amd/shard.py),
parses it with the oracle (the checker; the GPU path is covered by -m gpu),
and the per-rank records are gathered and compared with the single-process
parse of the whole batch. Also checks bench.py's max-over-ranks timing
reduction and weak-scaling packet numbering (rank r parses packets
r*n .. r*n+n-1 of the global generator stream)."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        zp = importlib.import_module("zero-packet_amd")
        import oracle as orc
        # mixed workload (IPv4/IPv6, IP-in-IP, IMIX sizes) with a few corrupt frames
        arena, offs, lens = zp.batch.generate_host("c5", 3000)
        arena[int(offs[7]) + 30] ^= 0xFF
        arena[int(offs[2500] + lens[2500]) - 1] ^= 0x01
        sub, o, ln, (lo, hi) = zp.shard.rank_shard(arena, offs, lens, rank, world)
        rec, ext = orc.parse_batch(sub, o, ln, 1)
        mine = torch.from_numpy(np.frombuffer(rec.tobytes() + ext.tobytes(), np.uint8).copy())
        parts = [None] * world
        dist.all_gather_object(parts, (lo, hi, rec.tobytes(), ext[0].tobytes(), ext[1].tobytes()))
        # bench.py's reduction: the slowest rank defines the step time
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # weak scaling: rank r's generator packets are r*n .. r*n+n-1
        n = 200
        a_r, o_r, l_r = zp.batch.generate_host("c3", n, first=rank * n)
        segs = [None] * world
        dist.all_gather_object(segs, bytes(a_r[:int(o_r[-1] + l_r[-1])]))
        dist.barrier()
        if rank == 0:
            q.put(("ok", parts, float(t.item()), segs, int(mine.numel())))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e)))
        raise


def test_shard_bounds_balance():
    zp = importlib.import_module("zero-packet_amd")
    lens = np.array([64, 1500, 64, 64, 1500, 700, 64, 1500], dtype=np.uint32)
    for world in (1, 2, 3, 4, 8):
        b = zp.shard.shard_bounds(lens, world)
        assert b[0] == 0 and b[-1] == lens.size and all(x <= y for x, y in zip(b, b[1:]))
    assert zp.shard.shard_bounds(np.zeros(0, np.uint32), 4) == [0, 0, 0, 0, 0]
    rng = np.random.default_rng(1)
    lens = rng.integers(64, 1501, 100000).astype(np.uint32)
    b = zp.shard.shard_bounds(lens, 8)
    per = [int(lens[b[r]:b[r + 1]].astype(np.int64).sum()) for r in range(8)]
    assert max(per) - min(per) <= 2 * 1500


def test_local_shard_rebases_any_layout():
    zp = importlib.import_module("zero-packet_amd")
    offs = np.array([500, 100, 900, 100], dtype=np.uint64)   # unordered + duplicate
    lens = np.array([64, 80, 70, 80], dtype=np.uint32)
    b0, b1, o, ln = zp.shard.local_shard(offs, lens, 0, 4)
    assert (b0, b1) == (100, 970) and o.tolist() == [400, 0, 800, 0]


def test_world2_gloo_shards_match_single_process():
    import oracle as orc
    zp = importlib.import_module("zero-packet_amd")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        msg = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert msg[0] == "ok", msg
    _, parts, tmax, segs, _ = msg
    assert tmax == float(world)
    assert all(p.exitcode == 0 for p in procs)
    # union of the shards == single-process parse of the whole batch
    arena, offs, lens = zp.batch.generate_host("c5", 3000)
    arena[int(offs[7]) + 30] ^= 0xFF
    arena[int(offs[2500] + lens[2500]) - 1] ^= 0x01
    rec, ext = orc.parse_batch(arena, offs, lens, 1)
    assert parts[0][0] == 0 and parts[-1][1] == 3000
    assert all(parts[r][1] == parts[r + 1][0] for r in range(world - 1))
    assert b"".join(p[2] for p in parts) == rec.tobytes()
    assert b"".join(p[3] for p in parts) == ext[0].tobytes()    # outer chains
    assert b"".join(p[4] for p in parts) == ext[1].tobytes()    # ip_in_ip chains
    assert (rec["err"] != 0).sum() >= 2
    # per-rank weak-scaling shards are consecutive slices of one packet stream
    a, o, l = zp.batch.generate_host("c3", 400)
    assert segs[0] + segs[1] == bytes(a[:int(o[-1] + l[-1])])
