"""Hierarchical (node-aware) all-reduce and sync_dense_mode 1 (k-step node
parameter averaging, reference boxps_worker.cc:1191-1258) over gloo with 4
ranks laid out as 2 "nodes" x 2 GPUs."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from paddlebox_amd.parallel.dense import DenseArena, DenseSync, FlatSGD, HierarchicalAllReduce


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE="2")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        h = HierarchicalAllReduce()
        out = {"nodes": h.nodes, "local": h.local_size}
        for n in (1, 7, 64, 1001):  # padded and unpadded shard splits
            t = torch.arange(n, dtype=torch.float32) * (rank + 1) + rank
            h.allreduce_(t)
            want = torch.arange(n, dtype=torch.float32) * sum(r + 1 for r in range(world)) + sum(range(world))
            out[f"n{n}"] = float((t - want).abs().max())
        # k-step node averaging: after k local SGD steps every rank holds the mean
        torch.manual_seed(0)
        m = torch.nn.Linear(5, 3)
        arena = DenseArena(m.parameters(), torch.device("cpu"))
        sync = DenseSync(arena, "kstep_node", k=2)
        opt = FlatSGD(arena, lr=0.1)
        for step in range(2):
            g = torch.Generator().manual_seed(10 * rank + step)
            x = torch.randn(4, 5, generator=g)
            arena.zero_grad()
            m(x).pow(2).mean().backward()
            sync.apply(opt)
        flat = arena.flat.clone()
        allp = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        out["replicas_equal"] = max(float((p - flat).abs().max()) for p in allp)
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_hierarchical_allreduce_and_kstep_node():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 4, _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=30)
    for rank, out in res:
        assert isinstance(out, dict), out
        assert out["nodes"] == 2 and out["local"] == 2
        for k, v in out.items():
            if k.startswith("n") and k != "nodes":
                assert v == 0.0, (rank, k, v)
        assert out["replicas_equal"] < 1e-6


def _coll_worker(rank, world, port, q):
    try:
        import numpy as np

        import paddlebox_amd.fluid as fluid
        from paddlebox_amd.fluid.layers import collective as C

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE="2")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        main, startup = fluid.Program(), fluid.Program()
        with fluid.program_guard(main, startup), fluid.unique_name.guard():
            x = fluid.layers.data("x", shape=[3], dtype="float32", append_batch_size=False)
            y = fluid.layers.data("y", shape=[2], dtype="float32", append_batch_size=False)
            s = C._c_allreduce(x, reduce_type="sum")
            mx = C._c_allreduce(x, reduce_type="max")
            g = C._c_allgather(x, nranks=world)
            b = C._c_broadcast(x, root=1)
            m0 = C._c_mixallgather([x, y], nranks=2, nccl_mode=0)
            m1 = C._c_mixallgather([x, y], nranks=2, nccl_mode=1)
            m2 = C._c_mixallgather([x, y], nranks=2, nccl_mode=2)
            xs = C._c_allreduce_xsum([x, y])
        exe = fluid.Executor(fluid.CPUPlace())
        feed = {"x": np.array([rank, rank + 1, 10 * rank], np.float32), "y": np.array([1, rank], np.float32)}
        outs = exe.run(main, feed=feed, fetch_list=[s, mx, g, b, m0, m1, m2] + xs)
        q.put((rank, [np.asarray(o).reshape(-1).tolist() for o in outs]))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))


def test_fluid_collective_ops_four_ranks():
    """c_allreduce_{sum,max}, c_allgather, c_broadcast, c_mixallgather
    (modes 0/1/2, 2 nodes x 2 ranks) and c_allreduce_xsum inside a program."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 4, _port()
    ps = [ctx.Process(target=_coll_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    xs = [[r, r + 1, 10 * r] for r in range(world)]
    ys = [[1, r] for r in range(world)]
    cat = [x + y for x, y in zip(xs, ys)]
    tot = [sum(c[i] for c in cat) for i in range(5)]
    node = [[sum(cat[r][i] for r in (2 * n, 2 * n + 1)) for i in range(5)] for n in range(2)]
    for r in range(world):
        out = res[r]
        assert not isinstance(out, str), out
        s, mx, g, b, m0, m1, m2, xsum, ysum = out
        assert s == [6, 10, 60] and mx == [3, 4, 30]
        assert g == sum(xs, []) and b == xs[1]
        assert m0 == tot and m1 == node[0] + node[1] and m2 == sum(cat, [])
        assert xsum == [6, 10, 60] and ysum == [4, 6]
