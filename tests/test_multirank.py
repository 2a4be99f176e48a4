"""CPU, world_size 2 (gloo): the N>1 path of bench.py — contiguous / byte-balanced
shards, per-rank outputs that concatenate to the single-GPU result, and the
max-over-ranks timing reduction.  The per-rank checksum here is the oracle
(CPU stand-in for each GPU's engine call); the GPU path itself is the same
call on the rank's own shard."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch

    from oracle import oracle as orc
    from tcpip_network_protocol_stack_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        # fixed-stride batch: 10001 x 1500 B of the NS spec stream
        n, L, seed = 10001, 1500, 0x10710000
        sh = shard.fixed_stride_shard(n, L, L, rank, WORLD)
        data = orc.fill_bytes(seed, sh.byte0, sh.nbytes)
        init = orc.pseudo_inits(seed, sh.n, length=L, index0=sh.index0)
        out = orc.checksum_batch(data, sh.n, stride=L, seg_len=L, init=init)
        parts = [None] * WORLD
        dist.all_gather_object(parts, (sh.index0, out.tolist()))
        # mixed batch: byte-balanced cuts of the packed offsets
        m, seed4 = 3000, 0x10710004
        lens = np.array([orc.mixed_len(seed4, i) for i in range(m)], dtype=np.uint64)
        off = np.zeros(m + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        ms = shard.offsets_shard(off, rank, WORLD)
        d4 = orc.fill_bytes(seed4, ms.byte0, ms.nbytes)
        o4 = orc.checksum_batch(d4, ms.n, offsets=off[ms.index0:ms.index0 + ms.n + 1] - off[ms.index0])
        parts4 = [None] * WORLD
        dist.all_gather_object(parts4, (ms.index0, o4.tolist(), ms.nbytes))
        t = shard.max_over_ranks(0.25 + rank, dist)
        # bench.py's self-check at N > 1: the ranks' u16 outputs gathered in
        # rank order over gloo, and one row per rank
        import bench

        whole = bench.gather_u16(torch.from_numpy(out.view(np.int16)), dist)
        rows = bench.gather_rows({"rank": rank, "segments": sh.n}, dist)
        if rank == 0:
            q.put((parts, parts4, t, bench.sha256_u16(whole), rows))
        else:
            assert whole is None and rows is None
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_concatenate_to_single_gpu_result(orc):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    parts, parts4, tmax, whole_sha, rows = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # fixed stride
    n, L, seed = 10001, 1500, 0x10710000
    full = orc.checksum_batch(orc.fill_bytes(seed, 0, n * L), n, stride=L, seg_len=L,
                              init=orc.pseudo_inits(seed, n, length=L))
    got = [x for _, o in sorted(parts) for x in o]
    assert got == full.tolist()
    import hashlib

    assert whole_sha == hashlib.sha256(full.astype(np.uint16).tobytes()).hexdigest()
    assert [r["rank"] for r in rows] == [0, 1] and sum(r["segments"] for r in rows) == n
    # mixed, byte balanced
    m, seed4 = 3000, 0x10710004
    lens = np.array([orc.mixed_len(seed4, i) for i in range(m)], dtype=np.uint64)
    off = np.zeros(m + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    full4 = orc.checksum_batch(orc.fill_bytes(seed4, 0, int(off[-1])), m, offsets=off)
    got4 = [x for _, o, _ in sorted(parts4) for x in o]
    assert got4 == full4.tolist()
    nb = [b for _, _, b in parts4]
    assert abs(nb[0] - nb[1]) <= 65536  # within one segment of equal bytes
    assert tmax == pytest.approx(1.25)


def test_shard_ranges_cover_exactly():
    from tcpip_network_protocol_stack_amd import shard

    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    off = np.cumsum([0] + [100] * 10 + [10000] + [100] * 10).astype(np.uint64)
    cuts = shard.byte_balanced_cuts(off, 4)
    assert cuts[0] == 0 and cuts[-1] == 21 and (np.diff(cuts) >= 0).all()
