"""Multi-rank exchange of self-play records on CPU with the gloo backend
(world size 2): packing round trip, variable-length all-gather in rank
order, weight broadcast, replay-buffer deque semantics."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hzamd.distributed import (ReplayBuffer, all_gather_records, broadcast_weights, pack_records, pi_of,
                               unpack_records)


def fake_records(rank, m):
    g = torch.Generator().manual_seed(100 + rank)
    states = torch.randint(-2**62, 2**62, (m, 6), generator=g, dtype=torch.int64)
    visits = torch.randint(0, 400, (m, 143), generator=g, dtype=torch.int32)
    z = torch.randint(-1, 2, (m,), generator=g).float()
    player = torch.randint(0, 2, (m,), generator=g)
    return states, visits, z, player


def test_pack_roundtrip():
    s, v, z, p = fake_records(0, 257)
    s2, v2, z2, p2 = unpack_records(pack_records(s, v, z, p))
    assert (s2 == s).all() and (v2 == v).all() and (z2 == z).all() and (p2 == p.to(torch.int8)).all()
    pi = pi_of(v)
    ref = (v.double() / v.double().sum(1, keepdim=True)).float()
    assert (pi == ref).all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = 5 + 7 * rank
        rec = pack_records(*fake_records(rank, m))
        allrec = all_gather_records(rec)
        expect = torch.cat([pack_records(*fake_records(r, 5 + 7 * r)) for r in range(world)])
        ok_gather = bool((allrec == expect).all())
        net = torch.nn.Linear(4, 3)
        with torch.no_grad():
            for p in net.parameters():
                p.fill_(float(rank + 1))
        broadcast_weights(net, src=0)
        ok_bcast = all(bool((p == 1.0).all()) for p in net.parameters())
        q.put((rank, ok_gather, ok_bcast, allrec.shape[0]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_all_gather_and_broadcast():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_g, ok_b, total in res:
        assert ok_g and ok_b and total == 5 + 12


def test_replay_buffer_keeps_newest():
    rb = ReplayBuffer(10, "cpu")
    data = pack_records(*fake_records(3, 25))
    rb.extend(data[:4])
    rb.extend(data[4:13])
    assert len(rb) == 10 and (rb.records() == data[3:13]).all()
    rb.extend(data[13:25])
    assert (rb.records() == data[15:25]).all()
