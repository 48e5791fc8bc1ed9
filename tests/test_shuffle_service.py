"""Native shuffle message service (boxps::PaddleShuffler contract,
data_set.cc:1906-1935,2440-2604) and the dataset's global shuffle over it.

* 3 in-process MsgService ranks: delivery, per-peer FIFO order (the empty
  end-of-stream message arrives after the data), ack callbacks, wait_done,
  loopback sends.
* 3 spawned processes (gloo rendezvous only for the endpoint exchange): every
  record ends on exactly one rank, on the rank its line-id / search-id hash
  names, with its feasigns and line id intact.
"""
import os
import socket
import threading

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from paddlebox_amd import _native

h = _native.host()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_msg_service_delivery_order_and_acks():
    W = 3
    svcs = [h.MsgService(r, W) for r in range(W)]
    eps = [f"127.0.0.1:{s.listen('127.0.0.1', 0)}" for s in svcs]
    ts = [threading.Thread(target=s.connect, args=(eps,)) for s in svcs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    got = {r: [] for r in range(W)}
    lock = threading.Lock()

    def handler(r):
        def on_receive(src, data):
            with lock:
                got[r].append((src, bytes(data)))
        return on_receive

    sids = [s.register_handler(handler(r)) for r, s in enumerate(svcs)]
    assert len(set(sids)) == 1  # same registration order -> same service id
    sid = sids[0]
    acks = []
    for r, s in enumerate(svcs):
        for d in range(W):
            for k in range(5):
                s.send_message((sid << 16) | d, f"{r}->{d}#{k}".encode() * (k * 1000 + 1),
                               lambda r=r: acks.append(r))
            s.send_message((sid << 16) | d, b"")  # end marker
    for s in svcs:
        s.wait_done(sid)
    assert len(acks) == W * W * 5
    for d in range(W):
        for src in range(W):
            msgs = [m for (s_, m) in got[d] if s_ == src]
            assert len(msgs) == 6 and msgs[-1] == b""  # FIFO: end marker last
            for k in range(5):
                assert msgs[k] == f"{src}->{d}#{k}".encode() * (k * 1000 + 1)
    assert sum(s.bytes_sent() for s in svcs) > 0
    for s in svcs:
        s.unregister_consumer(sid)
        s.destroy()


SLOTS = [("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1)]


def _records(rank, n):
    lines = []
    for i in range(n):
        ins = f"{rank:02d}{i:030d}"
        k = rank * 100000 + i + 1
        lines.append(f"1 {ins} 1 {i % 2} 2 {k} {k + 5000000}")
    return lines


def _make_ds(rank, world, n):
    from paddlebox_amd.data.dataset import PadBoxSlotDataset

    ds = PadBoxSlotDataset(rank=rank, world=world)
    ds._native.set_slots([h.SlotDesc(*s) for s in SLOTS])
    pc = h.ParseConfig()
    pc.parse_ins_id = True
    ds._native.set_parse(pc)
    ds._configured = True
    assert ds.add_lines(_records(rank, n)) == n
    return ds


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ds = _make_ds(rank, world, 200 + 37 * rank)
        if mode == "lineid":
            ds.set_merge_by_lineid(True)
        got = ds.global_shuffle(seed=3, chunk=17)
        ids = ds._native.ins_ids()
        keys, lod, _ = ds._native.build_batch(0, ds.get_memory_data_size(), False)
        q.put((rank, got, ids, keys.tolist(), lod.tolist()))
    finally:
        dist.barrier()
        from paddlebox_amd.data import shuffler

        shuffler.finalize()
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["random", "lineid"])
def test_global_shuffle_three_ranks(mode):
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got, ids, keys, lod = q.get(timeout=120)
        res[r] = (got, ids, keys, lod)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    all_ids = [i for r in range(world) for i in res[r][1]]
    expect = [f"{r:02d}{i:030d}" for r in range(world) for i in range(200 + 37 * r)]
    assert sorted(all_ids) == sorted(expect)  # nothing lost, nothing duplicated
    assert sum(res[r][0] for r in range(world)) > 0  # records did move
    for r in range(world):
        got, ids, keys, lod = res[r]
        # the batch is built in the dataset's (shuffled) order; map each record's
        # line id -> its two feasigns and check they travelled together
        order = [int(i[2:]) + 100000 * int(i[:2]) + 1 for i in ids]
        assert sorted(k for k in keys if k < 5000000) == sorted(order)
        assert sorted(k - 5000000 for k in keys if k >= 5000000) == sorted(order)
        if mode == "lineid":
            for i in ids:
                assert h.xxh64(i[:32], 0) % world == r


def _kill_worker(rank, W, q_in, q_out):
    import os as _os

    from paddlebox_amd import _native as nat

    hh = nat.host()
    svc = hh.MsgService(rank, W)
    q_out.put(("port", rank, svc.listen("127.0.0.1", 0)))
    eps = q_in.get(timeout=60)
    svc.connect(eps, 30.0)
    seen = [0]

    def on_receive(src, data):
        seen[0] += 1
        if rank == W - 1 and seen[0] == 3:  # the victim dies abruptly mid-shuffle
            _os._exit(3)

    sid = svc.register_handler(on_receive)
    err = None
    try:
        for k in range(200):
            for d in range(W):
                if d != rank:
                    svc.send_message((sid << 16) | d, b"x" * 65536)
        for d in range(W):
            if d != rank:
                svc.send_message((sid << 16) | d, b"")
        svc.wait_done(sid)
    except RuntimeError as e:
        err = str(e)
    q_out.put(("done", rank, err, list(svc.broken_peers())))
    svc.unregister_consumer(sid)
    svc.destroy()


def test_msg_service_lost_peer_fails_fast():
    """a peer that dies mid-shuffle must fail the survivors'
    wait_done with an error naming it, not hang them forever."""
    import time

    W = 3
    ctx = mp.get_context("spawn")
    q_in = [ctx.Queue() for _ in range(W)]
    q_out = ctx.Queue()
    ps = [ctx.Process(target=_kill_worker, args=(r, W, q_in[r], q_out)) for r in range(W)]
    for p in ps:
        p.start()
    ports = {}
    while len(ports) < W:
        kind, r, port = q_out.get(timeout=60)
        ports[r] = port
    eps = [f"127.0.0.1:{ports[r]}" for r in range(W)]
    for q in q_in:
        q.put(eps)
    t0 = time.time()
    res = {}
    while len(res) < W - 1:
        kind, r, err, broken = q_out.get(timeout=90)
        res[r] = (err, broken)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert ps[W - 1].exitcode == 3
    for r in range(W - 1):
        err, broken = res[r]
        assert err is not None and "rank 2" in err, res
        assert W - 1 in broken, res
    assert time.time() - t0 < 60
