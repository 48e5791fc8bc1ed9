"""Dense-sync modes over gloo with 2 ranks: transpiler GradAllReduce /
LocalSGD / MultiThread(all_gather), fleet sharding (ZeRO-1), checked against
a single-process reference of the same global batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from paddlebox_amd.parallel.dense import DenseArena, DenseSync, FlatAdam
from paddlebox_amd.parallel.sharding import ShardedFlatAdam


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 1))


def _data(step, rank, world):
    g = torch.Generator().manual_seed(100 + step)
    x = torch.randn(8 * world, 6, generator=g)
    y = torch.randn(8 * world, 1, generator=g)
    return x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]


def _train(mode, rank, world, steps=4):
    m = _model()
    arena = DenseArena(m.parameters(), torch.device("cpu"))
    if mode == "sharding":
        opt = ShardedFlatAdam(arena, lr=0.05)
        sync = DenseSync(arena, "none")
    else:
        opt = FlatAdam(arena, lr=0.05)
        sync = DenseSync(arena, mode)
    for s in range(steps):
        x, y = _data(s, rank, world)
        arena.zero_grad()
        ((m(x) - y) ** 2).mean().backward()
        sync.apply(opt)
    return arena.flat.clone()


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _train(mode, rank, world).detach().numpy()))  # by value: no fd sharing with an exiting worker
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _run(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {r: torch.from_numpy(v) for r, v in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(timeout=60)
    return out


def _single_process_reference(world=2, steps=4):
    """grad_allreduce semantics: mean of the per-rank gradients each step."""
    m = _model()
    arena = DenseArena(m.parameters(), torch.device("cpu"))
    opt = FlatAdam(arena, lr=0.05)
    for s in range(steps):
        acc = torch.zeros_like(arena.grad)
        for r in range(world):
            x, y = _data(s, r, world)
            arena.zero_grad()
            ((m(x) - y) ** 2).mean().backward()
            acc += arena.grad
        arena.grad.copy_(acc)
        opt.step(1.0 / world)
    return arena.flat.clone()


@pytest.mark.parametrize("mode", ["grad_allreduce", "sharding"])
def test_allreduce_and_zero1_match_reference(mode):
    out = _run(mode)
    ref = _single_process_reference()
    for r in (0, 1):
        torch.testing.assert_close(out[r], ref, rtol=1e-5, atol=1e-6)


def test_allgather_and_local_sgd_keep_replicas_identical():
    for mode in ("allgather", "local_sgd"):
        out = _run(mode)
        torch.testing.assert_close(out[0], out[1], rtol=0, atol=0)


def test_transpilers_and_fleet_record_modes():
    import paddlebox_amd.fluid as fluid
    from paddlebox_amd import fleet as fleet_mod

    prog, start = fluid.Program(), fluid.Program()
    fluid.transpiler.GradAllReduce().transpile(start, prog, 0, "127.0.0.1:1,127.0.0.1:2", "127.0.0.1:1")
    assert prog._collective["mode"] == "grad_allreduce" and prog._collective["nranks"] == 2
    assert prog._collective["rewritten"]
    fluid.transpiler.LocalSGD().transpile(start, prog, 1, ["a:1", "b:2"], "b:2")
    assert prog._collective["mode"] == "local_sgd" and prog._collective["rank"] == 1
    fluid.transpiler.MultiThread(trans_mode="all_gather").transpile(start, prog, 0, "a:1", "a:1")
    assert prog._collective["mode"] == "allgather"
    st = fleet_mod.DistributedStrategy()
    st.sharding = True
    with fluid.program_guard(prog, start):
        x = fluid.layers.data(name="x", shape=[4], dtype="float32")
        loss = fluid.layers.reduce_mean(fluid.layers.fc(x, 1))
        fleet_mod.fleet.distributed_optimizer(fluid.optimizer.Adam(0.01), st).minimize(loss)
    assert prog._collective["mode"] == "sharding"
    prog2, start2 = fluid.Program(), fluid.Program()
    with fluid.program_guard(prog2, start2):
        x = fluid.layers.data(name="x", shape=[4], dtype="float32")
        loss = fluid.layers.reduce_mean(fluid.layers.fc(x, 1))
        fleet_mod.fleet.distributed_optimizer(fluid.optimizer.Adam(0.01), fleet_mod.DistributedStrategy()).minimize(loss)
    types = [op.type for op in prog2.global_block().ops]
    assert prog2._collective["mode"] == "grad_allreduce" and types.count("c_allreduce_sum") == 1
    assert "coalesce_tensor" in types
