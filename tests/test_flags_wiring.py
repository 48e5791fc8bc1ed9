"""PaddleBox flags that change behaviour: instance shuffle,
filelist polling, k-step moment sync, metrics debug print."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from paddlebox_amd.data.dataset import PadBoxSlotDataset, SlotVar
from paddlebox_amd.utils.flags import set_flags


def _ds(n=50):
    ds = PadBoxSlotDataset(rank=1, world=2)
    ds.set_use_var([SlotVar("label", "int64", (1,), 0), SlotVar("s0", "int64", (1,), 1)])
    ds.set_batch_size(10)
    ds.add_lines([f"1 {i % 2} 1 {i + 1}" for i in range(n)])
    return ds


def test_ins_shuffle_and_polling_flags():
    ds = _ds()
    ds.set_filelist([f"f{i}" for i in range(6)])
    assert ds._my_files() == ["f1", "f3", "f5"]  # rank-strided
    set_flags({"FLAGS_padbox_dataset_disable_polling": True, "FLAGS_padbox_disable_ins_shuffle": True})
    try:
        assert ds._my_files() == [f"f{i}" for i in range(6)]
        ds.prepare_train(shuffle=None)
        assert ds._native.order().tolist() == list(range(50))  # no per-pass shuffle
    finally:
        set_flags({"FLAGS_padbox_dataset_disable_polling": False, "FLAGS_padbox_disable_ins_shuffle": False})
    ds.prepare_train(shuffle=None)
    assert ds._native.order().tolist() != list(range(50))


def test_metrics_debug_print(caplog):
    from paddlebox_amd.metrics.registry import MetricRegistry

    reg = MetricRegistry(None)
    reg.init_metric("AucCalculator", "auc", "label", "pred", bucket_size=1000)
    reg.add_batch({"label": torch.tensor([0.0, 1.0, 1.0, 0.0]), "pred": torch.tensor([0.1, 0.9, 0.6, 0.4])})
    set_flags({"FLAGS_enable_debug_print_metrics_info": True})
    try:
        with caplog.at_level("INFO", logger="pbx"):
            msg = reg.get_metric_msg("auc")
    finally:
        set_flags({"FLAGS_enable_debug_print_metrics_info": False})
    assert msg[0] == 1.0 and msg[7] == 4
    assert any("metric auc" in r.getMessage() for r in caplog.records)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _moment_worker(rank, world, port, q):
    try:
        from paddlebox_amd.parallel.dense import DenseArena, DenseSync, FlatAdam

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        set_flags({"FLAGS_enable_sync_dense_moment": True})
        torch.manual_seed(0)
        m = torch.nn.Linear(4, 2)
        arena = DenseArena(m.parameters(), torch.device("cpu"))
        opt = FlatAdam(arena, lr=0.1)
        sync = DenseSync(arena, "kstep", k=2)
        for step in range(2):
            g = torch.Generator().manual_seed(rank * 10 + step)
            arena.zero_grad()
            m(torch.randn(3, 4, generator=g)).pow(2).sum().backward()
            sync.apply(opt)
        outs = [torch.empty_like(opt.m) for _ in range(world)]
        dist.all_gather(outs, opt.m.clone())
        q.put((rank, max(float((o - opt.m).abs().max()) for o in outs)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_kstep_moment_sync_flag():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_moment_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=30)
    for rank, v in res:
        assert not isinstance(v, str), v
        assert v < 1e-7  # the Adam moments were averaged with the parameters
