"""Multi-rank sharding rehearsed on CPU with gloo, world_size 2:
each rank encodes only its contiguous row-group shard (as bench.py does),
decodes it with the oracle, and the concatenation over ranks must equal the
single-rank full table -- no data-path collective, only the checksum gather
and the MAX reduction bench.py uses for timing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bench import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digests(rf):
    import hashlib
    out = []
    for c in range(rf.ncols):
        raw = rf.decode_column(c, 2)
        data = b"\0".join(rf.strings(raw)) if rf.column(c)[1] in (20, 21) else raw.tobytes()
        out.append(hashlib.sha1(data).hexdigest())
    return out


def _worker(rank, world, port, wl, scale, nrows, q):
    try:
        _work(rank, world, port, wl, scale, nrows, q)
    except BaseException as e:  # surface child failures instead of hanging the parent
        q.put(("error", rank, repr(e)))
        raise


def _work(rank, world, port, wl, scale, nrows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pkgload
    from oracle import flsref
    fl = pkgload.load()
    total = fl.gen_nrows(wl, scale, nrows)
    nrg = (total + 65535) // 65536
    rg0, rg1 = shard_range(nrg, rank, world)
    img = fl.gen_image(wl, scale, nrows, rg0, rg1, 2)
    rf = flsref.RefFile(img)
    sums = _digests(rf)
    out = [None] * world
    dist.all_gather_object(out, (rg0, rg1, rf.f.row_offset, rf.nrows, sums))
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put(("ok", out, float(t.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("wl,scale,nrows", [("lineitem", 0.05, 0), ("c3", 1, 5 * 65536 + 7)])
def test_two_rank_shards_cover_table(_built, wl, scale, nrows):
    ctx = mp.get_context("fork")  # children never touch a GPU
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, wl, scale, nrows, q)) for r in range(2)]
    for p in procs:
        p.start()
    msg = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert msg[0] == "ok", msg
    _, out, tmax = msg
    assert all(p.exitcode == 0 for p in procs)
    assert tmax == 2.0
    import pkgload
    from oracle import flsref
    fl = pkgload.load()
    total = fl.gen_nrows(wl, scale, nrows)
    nrg = (total + 65535) // 65536
    (a0, a1, off0, n0, s0), (b0, b1, off1, n1, s1) = out
    assert (a0, a1, b0, b1) == (0, nrg // 2, nrg // 2, nrg)
    assert off0 == 0 and off1 == a1 * 65536 and n0 + n1 == total
    # each rank's shard decodes exactly like its rows of one full-table image
    import hashlib
    full = flsref.RefFile(fl.gen_image(wl, scale, nrows, 0, nrg, 2))
    for (r0, r1, sums) in [(a0, a1, s0), (b0, b1, s1)]:
        lo, hi = r0 * 65536, min(total, r1 * 65536)
        exp = []
        for c in range(full.ncols):
            raw = full.decode_column(c, 2)
            w = full.out_width(c)
            part = raw[lo * w:hi * w]
            data = b"\0".join(full.strings(part)) if full.column(c)[1] in (20, 21) else part.tobytes()
            exp.append(hashlib.sha1(data).hexdigest())
        assert exp == sums


def test_shard_range_partitions():
    for nrg in (1, 2, 7, 92, 9156):
        for world in (1, 2, 4, 8):
            r = [shard_range(nrg, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == nrg
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
