"""dlopen instance-parser plugins (csrc/host/parser_plugin.h; reference
ISlotParser ABI fw/data_feed.h:1964-2015, loader data_feed.cc:3604-3670),
exercised with the shipped Criteo TSV plugin (csrc/plugins/)."""
import math
import os
import subprocess

import pytest
import torch

from paddlebox_amd import _native
from paddlebox_amd.data.dataset import PadBoxSlotDataset, SlotVar

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def plugin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("plug") / "criteo_tsv_parser.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "csrc", "host"),
                    os.path.join(ROOT, "csrc", "plugins", "criteo_tsv_parser.cc"), "-o", out], check=True)
    return out


def _line(label, ints, cats):
    return "\t".join([str(label)] + [("" if v is None else str(v)) for v in ints] + [c or "" for c in cats])


def test_native_dataset_with_plugin(plugin):
    h = _native.host()
    slots = [h.SlotDesc("label", "uint64", True, True, 1), h.SlotDesc("dense", "float", True, True, 13)]
    slots += [h.SlotDesc(f"C{i}", "uint64", True, False, 1) for i in range(1, 27)]
    slots += [h.SlotDesc("I3", "float", False, True, 1)]  # unused slot: values discarded
    d = h.SlotDataset()
    d.set_slots(slots)
    d.set_so_parser(plugin)
    assert d.has_so_parser()
    cats = ["%08x" % (0x1000 + i) for i in range(26)]
    cats2 = list(cats)
    cats2[5] = None  # empty categorical -> no feasign in C6
    lines = [_line(1, [3] + [None] * 12, cats), _line(0, list(range(13)), cats2),
             "garbage line", _line(0, [None] * 13, [None] * 26)]  # last: no sparse feasign -> dropped
    assert d.add_lines(lines) == 2
    assert d.bad_lines() == 2
    keys, lod, dense = d.build_batch(0, 2, False)
    assert keys.numel() == 26 + 25
    assert int(lod.view(26, 3)[5, 2] - lod.view(26, 3)[5, 1]) == 0
    assert dense[:, 0].tolist() == [1.0, 0.0]  # label column first
    assert dense[0, 1].item() == pytest.approx(math.log1p(3))
    torch.testing.assert_close(dense[1, 1:], torch.log1p(torch.arange(13.0)))
    # the same categorical value in the same slot hashes to the same key, different slots differ
    k = keys.tolist()
    assert k[0] == k[1] and len(set(k[::2])) == 26


def test_padbox_dataset_so_parser(plugin, tmp_path):
    f = tmp_path / "part-0.tsv"
    cats = ["%08x" % (0x2000 + i) for i in range(26)]
    f.write_text("\n".join(_line(i % 2, [i] * 13, cats) for i in range(20)) + "\n")
    ds = PadBoxSlotDataset(rank=0, world=1)
    ds.set_use_var([SlotVar("label", "int64", (1,), 0), SlotVar("dense", "float32", (13,), 0)]
                   + [SlotVar(f"C{i}", "int64", (1,), 1) for i in range(1, 27)])
    ds.set_so_parser_name(plugin)
    ds.set_filelist([str(f)])
    ds.set_batch_size(8)
    ds.load_into_memory(register_keys=False)
    assert len(ds) == 20
    b = ds.build_batch(0, 8)
    assert b.keys.numel() == 8 * 26
