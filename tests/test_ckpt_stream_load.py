"""Streaming, per-rank batch-model load (VERDICT r3 #6b; reference: the PS loads
``model_path`` per node, box_wrapper.cc:1201-1242).

Parts are memory-mapped and walked in chunks much smaller than the model
here (ckpt.LOAD_CHUNK_ROWS), so a rank never holds more than ~2 chunks:
* a model saved by one rank, loaded by 2 gloo ranks: each rank reads every
  other part (here: rank 0 the only part, rank 1 none) and the rows reach
  their owners through the bounded per-round all-to-all;
* a model saved by 2 owner-sharded ranks (meta "world" = 2), loaded by 2
  ranks: each reads only its own part.
Every rank must end with exactly the rows it owns, bit-identical."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps import checkpoint as ckpt
from paddlebox_amd.ps.config import SparseSGDConfig
from paddlebox_amd.ps.cpu_table import CpuSparseTable

N, DIM = 5000, 8


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model_rows():
    g = torch.Generator().manual_seed(3)
    keys = torch.unique(torch.randint(1, 1 << 62, (N,), generator=g))
    h = ref.mix64(keys)
    t = CpuSparseTable(DIM)
    t.insert_mixed(h, SparseSGDConfig(), init_embedx=True)
    k, v = t.export(True)
    v = torch.rand(v.shape, generator=g)
    t.assign(k, v)
    return t


def _save(root):
    t = _model_rows()
    ckpt.save_batch_model(t, os.path.join(root, "w1"), 0)  # one part, no world in meta
    h, v = t.export(True)
    for r in range(2):  # owner-sharded parts of a 2-rank job
        m = ref.owner_of(h, 2) == r
        part = CpuSparseTable(DIM)
        part.insert_mixed(h[m], SparseSGDConfig())
        part.assign(h[m], v[m])
        ckpt.save_batch_model(part, os.path.join(root, "w2"), r, world=2)
    return h, v


def _worker(rank, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from paddlebox_amd.ps.box_wrapper import BoxWrapper

        ckpt.LOAD_CHUNK_ROWS = 300  # ~17 chunks: rounds of 150 rows per rank
        out = {}
        for name in ("w1", "w2"):
            BoxWrapper._instance = None
            box = BoxWrapper(DIM, device="cpu")
            box.initialize_gpu_and_load_model(slot_vector=[1], max_keys=1000)
            n = box.load_model(os.path.join(root, name))
            h, v = box.engine.table.export(True)
            # numpy, not torch: a torch tensor crosses the queue as a shared fd
            # served by this process (gone once it exits)
            out[name] = (n, h.numpy(), v.numpy())
        q.put((rank, out))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_streamed_per_rank_load_routes_rows_to_owners(tmp_path):
    root = str(tmp_path)
    h, v = _save(root)
    assert ckpt.read_meta(os.path.join(root, "w2"))["world"] == 2
    assert "world" not in ckpt.read_meta(os.path.join(root, "w1"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, root, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    res = {r: {k: (n, torch.from_numpy(a), torch.from_numpy(b)) for k, (n, a, b) in o.items()} for r, o in res.items()}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    order = torch.argsort(h)
    for name in ("w1", "w2"):
        hs, vs, total = [], [], 0
        for r in range(2):
            n, hr, vr = res[r][name]
            assert n == hr.numel()
            assert bool((ref.owner_of(hr, 2) == r).all()), (name, r)
            hs.append(hr)
            vs.append(vr)
            total += n
        assert total == h.numel()
        ha, va = torch.cat(hs), torch.cat(vs)
        o = torch.argsort(ha)
        assert torch.equal(ha[o], h[order])
        torch.testing.assert_close(va[o], v[order], rtol=0, atol=0)


def test_part_chunks_are_memory_mapped(tmp_path):
    """iter_part_chunks walks a part in chunks of the requested size."""
    t = _model_rows()
    ckpt.save_batch_model(t, str(tmp_path), 0)
    sizes = [k.shape[0] for k, _ in ckpt.iter_part_chunks(str(tmp_path), 0, 777)]
    assert sum(sizes) == t.size() and max(sizes) == 777
    assert ckpt.list_parts(str(tmp_path)) == [0] and ckpt.part_rows(str(tmp_path), 0) == t.size()
    k0, v0 = next(ckpt.iter_part_chunks(str(tmp_path), 0, 10))
    assert k0.dtype == np.uint64 and v0.dtype == np.float32 and v0.shape[0] == 10
