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


@pytest.fixture(scope="module")
def side_plugin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("plug2") / "replica_index_parser.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "csrc", "host"),
                    os.path.join(ROOT, "csrc", "plugins", "replica_index_parser.cc"), "-o", out], check=True)
    return out


def test_replica_cache_and_input_index_feeds(side_plugin, tmp_path):
    """Replica-cache and input-index data feeds (reference
    SlotPaddleBoxDataFeedWithGpuReplicaCache / InputIndexDataFeed /
    InputTableDataFeed): the plugin appends each instance's cache vector to
    the pass's replica store and stores the row offset as a feasign; string
    keys resolve to input-table offsets while parsing."""
    from paddlebox_amd.ps.extras import GpuReplicaCache, InputTable

    h = _native.host()
    slots = [h.SlotDesc("label", "uint64", True, True, 1), h.SlotDesc("cache_off", "uint64", True, False, 1),
             h.SlotDesc("qidx", "uint64", True, False, 1), h.SlotDesc("s0", "uint64", True, False, 1),
             h.SlotDesc("s1", "uint64", True, False, 1)]
    d = h.SlotDataset()
    d.set_slots(slots)
    d.set_so_parser(side_plugin)
    idx_file = tmp_path / "index.txt"
    idx_file.write_text("kA 1 2 3\nkB 4 5 6\nkA 9 9 9\n")
    table = InputTable()
    assert d.load_index_files([str(idx_file)], table.native) == 3
    assert table.size() == 2 and table.get_offset("kB") == 1 and table.get_offset("kZ") == -1
    rep = h.ReplicaStore(4)
    d.set_replica_cache(rep)
    d.set_input_index(table.native)
    lines = ["1 kB 4 0.1 0.2 0.3 0.4 2 11 12 1 13", "0 kZ 3 1 2 3 1 21 1 22", "1 kA 4 5 6 7 8 1 31 1 32"]
    assert d.add_lines(lines) == 3
    keys, lod, dense = d.build_batch(0, 3, False)
    L = lod.view(4, 4)  # sparse slots: cache_off, qidx, s0, s1
    cache_keys = keys[int(L[0, 0]):int(L[0, 3])].tolist()
    assert sorted(cache_keys) == [0, 1, 2]
    rows = rep.data()
    assert rows.shape == (3, 4)
    want = {0: [0.1, 0.2, 0.3, 0.4], 1: [1, 2, 3, 0], 2: [5, 6, 7, 8]}  # short vector zero padded
    for i, off in enumerate(cache_keys):
        torch.testing.assert_close(rows[off], torch.tensor(want[i], dtype=torch.float32))
    # qidx: line 0 -> kB (1), line 1 -> kZ absent (no feasign), line 2 -> kA (0)
    assert [int(L[1, i + 1] - L[1, i]) for i in range(3)] == [1, 0, 1]
    assert keys[int(L[1, 0]):int(L[1, 3])].tolist() == [1, 0]
    # the BoxWrapper-side tables serve the rows: replica cache pull, lookup_input
    rc = GpuReplicaCache(4).load_native(rep)
    torch.testing.assert_close(rc.pull(torch.tensor(cache_keys), 4), rows[torch.tensor(cache_keys)])
    got = table.lookup(torch.tensor([1, 0, -1]), 3, "cpu")
    torch.testing.assert_close(got, torch.tensor([[4.0, 5, 6], [1, 2, 3], [0, 0, 0]]))


def test_replica_cache_feed_through_the_feed_pass(side_plugin, tmp_path):
    """FLAGS_use_gpu_replica_cache: the feed pass gives the loader a fresh
    replica store; at EndFeedPass the box's replica cache holds its rows."""
    import paddlebox_amd.fluid as fluid
    from paddlebox_amd.ps.box_wrapper import BoxWrapper
    from paddlebox_amd.utils.flags import set_flags

    f = tmp_path / "part-0.txt"
    f.write_text("\n".join(f"{i % 2} k{i} 4 {i} {i + 1} {i + 2} {i + 3} 1 {100 + i} 1 {200 + i}"
                           for i in range(10)) + "\n")
    box = fluid.core.BoxWrapper(8, device="cpu", new=True)
    set_flags({"FLAGS_use_gpu_replica_cache": True, "FLAGS_gpu_replica_cache_dim": 4})
    try:
        box.initialize_gpu_and_load_model(slot_vector=[0, 1, 2], max_keys=10000)
        ds = PadBoxSlotDataset(rank=0, world=1)
        ds.set_use_var([SlotVar("label", "int64", (1,), 0), SlotVar("cache_off", "int64", (1,), 1),
                        SlotVar("s0", "int64", (1,), 1), SlotVar("s1", "int64", (1,), 1)])
        ds.set_so_parser_name(side_plugin)
        ds.set_filelist([str(f)])
        ds.set_batch_size(5)
        ds.box = box
        ds.load_into_memory()
        assert len(box.replica_cache) == 10
        b = ds.build_batch(0, 10)
        offs = b.keys[:10]  # cache_off is the first sparse slot, one feasign per instance
        rows = box.replica_cache.pull(offs, 4)
        first = rows[:, 0].tolist()
        assert sorted(first) == [float(i) for i in range(10)]
        torch.testing.assert_close(rows[:, 1] - rows[:, 0], torch.ones(10))
    finally:
        set_flags({"FLAGS_use_gpu_replica_cache": False})
        BoxWrapper._instance = None


UNROLL_PLUGIN = r"""
// test plugin: lines "label k1 k2 ...": one instance with all keys in slot 1;
// UnrollInstance splits every record into one instance per key
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "parser_plugin.h"
extern "C" {
void* pbx_parser_create(int, const char* const*, const char*) { return (void*)1; }
void pbx_parser_destroy(void*) {}
int pbx_parser_parse_line(void*, const char* line, size_t len, const pbx_ins_sink* s) {
  char buf[512];
  if (len >= sizeof(buf)) return -1;
  memcpy(buf, line, len); buf[len] = 0;
  char* p = buf;
  uint64_t lab = strtoull(p, &p, 10);
  s->add_u64(s->ctx, 0, &lab, 1);
  for (;;) {
    char* q;
    uint64_t k = strtoull(p, &q, 10);
    if (q == p) break;
    p = q;
    s->add_u64(s->ctx, 1, &k, 1);
  }
  char id[40];
  int n = snprintf(id, sizeof(id), "line-%llu", (unsigned long long)lab);
  s->set_meta(s->ctx, id, n, 0, 0, 0);
  return s->commit(s->ctx);
}
int64_t pbx_parser_unroll(void*, const pbx_record_view* v, const pbx_ins_sink* s) {
  int64_t out = 0;
  for (int64_t r = 0; r < v->n; ++r) {
    const uint64_t *lab, *keys;
    if (v->get_u64(v->ctx, r, 0, &lab) != 1) return -1;
    const int nk = v->get_u64(v->ctx, r, 1, &keys);
    for (int i = 0; i < nk; ++i) {
      s->add_u64(s->ctx, 0, lab, 1);
      s->add_u64(s->ctx, 1, &keys[i], 1);
      out += s->commit(s->ctx);
    }
  }
  return out;
}
}
"""


def test_unroll_instance_hook(tmp_path):
    """FLAGS_padbox_dataset_enable_unrollinstance + the plugin's optional
    pbx_parser_unroll (reference ISlotParser::UnrollInstance,
    data_feed.h:1994-1998, data_set.cc:2275-2277)."""
    from paddlebox_amd.utils.flags import set_flags

    src = tmp_path / "unroll.cc"
    src.write_text(UNROLL_PLUGIN)
    so = str(tmp_path / "unroll.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "csrc", "host"), str(src), "-o", so],
                   check=True)
    data = tmp_path / "part-0"
    data.write_text("1 11 12 13\n0 21\n1 31 32\n")

    def load(flag):
        set_flags({"FLAGS_padbox_dataset_enable_unrollinstance": flag})
        try:
            ds = PadBoxSlotDataset(rank=0, world=1)
            ds.set_use_var([SlotVar("label", "int64", (1,), 0), SlotVar("s", "int64")])
            ds.set_so_parser_name(so)
            ds.set_filelist([str(data)])
            ds.load_into_memory(register_keys=False)
            return ds
        finally:
            set_flags({"FLAGS_padbox_dataset_enable_unrollinstance": False})

    plain = load(False)
    assert plain.get_memory_data_size() == 3
    un = load(True)
    assert un.get_memory_data_size() == 6
    keys, lod, dense = un._native.build_batch(0, 6, False)
    assert keys.tolist() == [11, 12, 13, 21, 31, 32]
    assert lod.tolist() == [0, 1, 2, 3, 4, 5, 6]
    assert dense[:, 0].tolist() == [1, 1, 1, 0, 1, 1]


FILE_PLUGIN = r"""
// whole-file parser (ParseFileInstance): reads the stream through the host's
// read callback; lines "label k1 k2 ..."; the ins id is "<path>:<line no>"
// when the host passes the path
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include "parser_plugin.h"
extern "C" {
void* pbx_parser_create(int, const char* const*, const char*) { return (void*)1; }
void pbx_parser_destroy(void*) {}
int pbx_parser_parse_line(void*, const char*, size_t, const pbx_ins_sink*) { return -1; }
int64_t pbx_parser_parse_file(void*, const char* path, pbx_read_fn rd, void* rctx, const pbx_ins_sink* s) {
  std::string all;
  char buf[4096];
  int64_t n;
  while ((n = rd(rctx, buf, sizeof(buf))) > 0) all.append(buf, (size_t)n);
  int64_t out = 0, lineno = 0;
  size_t b = 0;
  while (b < all.size()) {
    size_t e = all.find('\n', b);
    if (e == std::string::npos) e = all.size();
    std::string ln = all.substr(b, e - b);
    b = e + 1;
    if (ln.empty()) continue;
    char* p = &ln[0];
    uint64_t lab = strtoull(p, &p, 10);
    s->add_u64(s->ctx, 0, &lab, 1);
    for (;;) {
      char* q;
      uint64_t k = strtoull(p, &q, 10);
      if (q == p) break;
      p = q;
      s->add_u64(s->ctx, 1, &k, 1);
    }
    std::string id = (path ? std::string(path) : std::string("-")) + ":" + std::to_string(lineno++);
    s->set_meta(s->ctx, id.data(), (int)id.size(), 0, 0, 0);
    out += s->commit(s->ctx);
  }
  return out;
}
}
"""


def test_whole_file_parser_mode(tmp_path):
    """FLAGS_enable_ins_parser_file (+ _add_file_path): the plugin's
    pbx_parser_parse_file reads whole files (reference ParseFileInstance,
    data_feed.cc:3850-3870)."""
    from paddlebox_amd.utils.flags import set_flags

    src = tmp_path / "fileparse.cc"
    src.write_text(FILE_PLUGIN)
    so = str(tmp_path / "fileparse.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "csrc", "host"), str(src), "-o", so],
                   check=True)
    f0 = tmp_path / "part-0"
    f0.write_text("1 11 12\n0 21\n")
    h = _native.host()
    set_flags({"FLAGS_enable_ins_parser_file": True, "FLAGS_enable_ins_parser_add_file_path": True})
    try:
        d = h.SlotDataset()
        d.set_slots([h.SlotDesc("label", "uint64", True, True, 1), h.SlotDesc("s", "uint64", True, False, 1)])
        pc = h.ParseConfig()
        pc.parse_ins_id = True
        d.set_parse(pc)
        d.set_so_parser(so)
        d.set_filelist([str(f0)])
        assert d.load_into_memory() == 2
        assert d.ins_ids() == [f"{f0}:0", f"{f0}:1"]
        keys, lod, dense = d.build_batch(0, 2, False)
        assert keys.tolist() == [11, 12, 21]
    finally:
        set_flags({"FLAGS_enable_ins_parser_file": False, "FLAGS_enable_ins_parser_add_file_path": False})
