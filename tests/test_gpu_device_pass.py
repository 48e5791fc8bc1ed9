"""Device-resident pass + on-device batch assembly (csrc/hip/batch_ops.hip)
against the native host builder (SlotDataset::build_batch), which the CPU
suite pins against the text parser."""
import numpy as np
import pytest
import torch

import paddlebox_amd.fluid as fluid
from paddlebox_amd.data.device_pass import DevicePass

pytestmark = pytest.mark.gpu

S, DENSE = 5, 3


def _lines(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        toks = ["1", str(int(rng.integers(0, 2)))]
        for s in range(S):
            k = int(rng.integers(1 if s == 0 else 0, 5))  # empty slots too
            toks += [str(k)] + [str(int(x)) for x in rng.integers(1, 1 << 62, size=k)]
        d = int(rng.integers(1, DENSE + 1))  # short dense rows are zero-padded
        toks += [str(d)] + [f"{x:.3f}" for x in rng.random(d)]
        out.append(" ".join(toks))
    return out


def _dataset(n=700):
    label = fluid.layers.data("label", shape=[1], dtype="int64")
    slots = [fluid.layers.data(f"slot{i}", shape=[1], dtype="int64", lod_level=1) for i in range(S)]
    dense = fluid.layers.data("dense", shape=[DENSE], dtype="float32")
    ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
    ds.set_use_var([label] + slots + [dense])
    ds.set_batch_size(64)
    ds.add_lines(_lines(n, 5))
    return ds


def test_device_assembly_matches_host_builder():
    dev = torch.device("cuda:0")
    with fluid.program_guard(fluid.Program(), fluid.Program()), fluid.unique_name.guard():
        ds = _dataset()
    nat = ds._native
    nat.shuffle(11)
    n = int(nat.size())
    dp = DevicePass(nat, dev)
    dp.set_order(nat.order())
    Dw = int(nat.dense_width())
    for b0, c in [(0, 100), (100, 64), (164, 1), (165, n - 165)]:
        kh, lh, dh = nat.build_batch(b0, c, False)
        L = kh.numel()
        keys = torch.full((L + 37,), 12345, dtype=torch.int64, device=dev)
        lod = torch.full((S * (c + 1),), -7, dtype=torch.int64, device=dev)
        den = torch.full((c, Dw), -7.0, device=dev)
        dp.assemble_sync(b0, c, keys, lod, den)
        torch.cuda.synchronize()
        assert torch.equal(keys[:L].cpu(), kh)
        assert bool((keys[L:] == -1).all())
        assert torch.equal(lod.cpu(), lh.view(-1))
        assert torch.equal(den.cpu(), dh.view(c, Dw))
        assert not dp.overflowed()
    # a key buffer smaller than the batch: flagged, nothing written past it
    kh, lh, dh = nat.build_batch(0, 100, False)
    buf = torch.full((kh.numel() + 64,), 99, dtype=torch.int64, device=dev)
    small = buf[: kh.numel() - 10]
    dp.assemble_sync(0, 100, small, torch.empty(S * 101, dtype=torch.int64, device=dev),
                     torch.empty(100, Dw, device=dev))
    torch.cuda.synchronize()
    assert dp.overflowed()
    assert bool((buf[kh.numel() - 10:] == 99).all())
    assert torch.equal(small.cpu(), kh[: kh.numel() - 10])
