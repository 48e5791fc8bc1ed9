"""IPC mesh collectives (csrc/hip/ipc.hip) across 2 processes.  The test box
has one GPU, so both ranks map each other's inboxes on the same device (the
same IPC handle path as across xGMI peers); results are checked against
the exact sums, eagerly and replayed from a captured HIP graph."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist

        from paddlebox_amd.parallel.ipc import IpcMesh

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        n = 5000
        mesh = IpcMesh(n * 4, device=dev, blocks=8)
        errs = []
        # inbox + flags in uncached device memory (hipExtMallocWithFlags), not
        # the caching allocator's coarse-grained hipMalloc memory
        from paddlebox_amd import _native

        unc = int(_native.hip().kIpcMallocUncached)
        for typ, d, flags in mesh.memory_attrs():
            errs.append(0.0 if (d == 0 and flags == unc) else 1000.0 + flags)
        for it in range(5):  # both parities, several epochs
            t = torch.arange(n, dtype=torch.float32, device=dev) * (rank + 1) + it
            mesh.allreduce_(t)
            want = torch.arange(n, dtype=torch.float32, device=dev) * sum(r + 1 for r in range(world)) + it * world
            errs.append(float((t - want).abs().max()))
        # fixed-slot all-to-all: slot p carries (rank, p, payload)
        sb = mesh.slot_bytes
        for it in range(3):
            send = torch.zeros(world, sb // 4, dtype=torch.int32, device=dev)
            for p in range(world):
                send[p, 0], send[p, 1], send[p, 2:10] = rank, p, it * 100 + rank * 10 + p
            recv = mesh.exchange(send).view(torch.int32).view(world, sb // 4).clone()
            for src in range(world):
                ok = int(recv[src, 0]) == src and int(recv[src, 1]) == rank and \
                    bool((recv[src, 2:10] == it * 100 + src * 10 + rank).all())
                errs.append(0.0 if ok else 1.0)
        # captured: the epoch advances on the device across replays
        buf = torch.zeros(n, dtype=torch.float32, device=dev)
        src = torch.full((n,), float(rank + 1), device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            buf.copy_(src)
            mesh.allreduce_(buf, average=True)
        torch.cuda.current_stream(dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            buf.copy_(src)
            mesh.allreduce_(buf, average=True)
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize(dev)
            errs.append(float((buf - (world + 1) / 2).abs().max()))
        dist.barrier()
        q.put((rank, errs, mesh.error()))
        mesh.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), True))


def test_ipc_mesh_allreduce_and_exchange_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    for rank, errs, err_flag in out:
        assert not isinstance(errs, str), errs
        assert not err_flag, f"rank {rank}: a wait timed out"
        assert max(errs) == 0.0, (rank, errs)


def _timeout_worker(rank, world, port, q):
    try:
        import torch.distributed as dist

        from paddlebox_amd.parallel.ipc import IpcMesh, IpcMeshError

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        mesh = IpcMesh(4096, device=dev, blocks=4, spin_limit=1 << 14)  # ~1 ms bound
        t = torch.ones(256, device=dev)
        mesh.allreduce_(t)  # both ranks: fine
        torch.cuda.synchronize(dev)
        ok_first = bool(torch.all(t == world)) and not mesh.error()
        if rank == 0:  # rank 1 never joins this one: rank 0 must time out, not hang
            mesh.allreduce_(t)
            torch.cuda.synchronize(dev)
        dist.barrier()
        poisoned = bool(torch.isnan(t).all()) if rank == 0 else True
        raised = False
        try:
            mesh.check()
        except IpcMeshError:
            raised = True
        q.put((rank, ok_first, poisoned, raised))
        mesh.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), False, False))


def test_ipc_mesh_lost_peer_times_out_and_poisons():
    """a wait that gives up must not let training continue on a
    stale slot: the sum is NaN, the error is sticky and check() raises."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    ps = [ctx.Process(target=_timeout_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict((o[0], o[1:]) for o in (q.get(timeout=180) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert out[0][0] is True and out[1][0] is True, out
    assert out[0][1] and out[0][2], out  # rank 0: NaN result, check() raised
    assert out[1][2] is False, out       # rank 1 saw no failure of its own
