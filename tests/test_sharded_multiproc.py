"""Full sharded DeepFM step over a real process group: W spawned processes
(gloo, one rank each) run the sparse engine sharded by key owner (key /
value / gradient all-to-all through TorchDistComm) plus the dense
grad all-reduce, and must end with the same dense parameters and sparse
table as ONE process training on the union of the rank batches.

The GPU build runs the same engine code path with RCCL (bench.py under
torchrun); on CPU the engine's sharded branch uses variable-split
all_to_all, which gloo provides."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from paddlebox_amd.data.synthetic import ragged_batch
from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.config import PSConfig

B, S, STEPS = 24, 4, 3


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(world):
    return [[ragged_batch(B, S, 3, 80, seed=1000 * step + r) for r in range(world)] for step in range(STEPS)]


def _cfg():
    cfg = PSConfig(embedx_dim=8)
    cfg.sgd.mf_create_thresholds = 0.0
    return cfg


def _model(engine):
    from paddlebox_amd.models.deepfm import DeepFM

    torch.manual_seed(0)
    return DeepFM(engine, num_slots=S, dense_dim=13, hidden=(16, 8), use_data_norm=False)


def _train(engine, model, batches_of_rank, sync=None):
    from paddlebox_amd.parallel.dense import DenseArena, DenseSync, FlatAdam

    arena = DenseArena(model.parameters(), torch.device("cpu"))
    opt = FlatAdam(arena, lr=1e-2)
    sync = sync or DenseSync(arena, "grad_allreduce")
    for b in batches_of_rank:
        engine.register_keys(b.keys, init_embedx=True)
        arena.zero_grad()
        loss, _ = model(b)
        loss.backward()
        sync.before_step()
        opt.step(sync.grad_scale())
    return arena.flat.clone()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from paddlebox_amd.ps.sparse_engine import SparseEngine

        eng = SparseEngine(_cfg(), max_keys=4096, device=torch.device("cpu"), capacity=20000)
        assert eng.sharded and eng.world == world
        model = _model(eng)
        batches = _batches(world)
        flat = _train(eng, model, [batches[s][rank] for s in range(STEPS)])
        h, v = eng.table.export(True)
        q.put((rank, flat.detach().numpy(), h.numpy(), v.detach().numpy()))  # by value: no fd sharing with an exiting worker
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _oracle(world):
    from paddlebox_amd.ps.sparse_engine import SparseEngine
    from tests.test_sharded_loopback import concat_batches

    eng = SparseEngine(_cfg(), max_keys=4096 * world, device=torch.device("cpu"), capacity=20000 * world)
    model = _model(eng)
    batches = _batches(world)
    union = [concat_batches(batches[s]) for s in range(STEPS)]

    class _NoSync:
        def before_step(self):
            pass

        def grad_scale(self):
            return 1.0

    flat = _train(eng, model, union, sync=_NoSync())
    return flat, eng


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_deepfm_step_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, (torch.from_numpy(f), torch.from_numpy(h), torch.from_numpy(v)))
               for r, f, h, v in (q.get(timeout=240) for _ in ps))
    for p in ps:
        p.join(timeout=60)
    flat, eng = _oracle(world)
    for r in range(world):  # dense replicas identical and equal to the union-batch step
        torch.testing.assert_close(res[r][0], flat, rtol=2e-4, atol=2e-6)
    allh = torch.cat([res[r][1] for r in range(world)])
    allv = torch.cat([res[r][2] for r in range(world)])
    for r in range(world):  # every key lives on its owner shard only
        assert bool((ref.owner_of(res[r][1], world) == r).all())
    assert allh.numel() == torch.unique(allh).numel() == eng.table.size()
    exp = eng.table.read(allh)
    torch.testing.assert_close(allv[:, :14], exp[:, :14], rtol=2e-4, atol=2e-6)
