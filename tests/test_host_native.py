"""Native host runtime (_pbx_host): CPU PS, AUC calculator, slot dataset."""
import os

import numpy as np
import pytest
import torch

from paddlebox_amd import _native
from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.config import SparseSGDConfig, row_layout
from paddlebox_amd.ps.cpu_table import _cfg_list

h = _native.host()


def test_cpu_table_insert_probe_push_matches_reference():
    t = h.CpuTable(8, 8)
    keys = ref.mix64(torch.arange(1, 501, dtype=torch.int64))
    t.insert(keys, 0.0, 1e-4, 0, 1)
    assert t.size() == 500
    rows = t.probe(keys)
    assert (rows >= 0).all() and torch.unique(rows).numel() == 500
    assert (t.probe(ref.mix64(torch.arange(1000, 1010))) == -1).all()
    cfg = SparseSGDConfig(mf_create_thresholds=1e9)
    push = torch.zeros(500, 12)
    push[:, 0] = 3
    push[:, 1] = torch.randint(1, 5, (500,)).float()
    push[:, 2] = (torch.rand(500) < 0.3).float()
    push[:, 3:] = torch.randn(500, 9) * 0.1
    before = t.gather(rows)
    t.push_adagrad(rows, push, _cfg_list(cfg))
    after = t.gather(rows)
    exp = ref.adagrad_update(before, push, 8, cfg)
    torch.testing.assert_close(after, exp, rtol=1e-5, atol=1e-6)


def test_cpu_table_shrink_and_save_filter():
    t = h.CpuTable(8, 4)
    l = row_layout(8)
    keys = ref.mix64(torch.arange(1, 11, dtype=torch.int64))
    t.insert(keys, 0.0, 0.0, 0, 1)
    rows = t.probe(keys)
    vals = t.gather(rows)
    vals[:5, 0] = 100.0  # shows
    vals[:5, 1] = 10.0
    vals[:3, l["delta_score"]] = 1.0
    t.assign(rows, vals)
    f = h.SaveFilter()
    k, v = t.select_for_save(1, f)  # delta
    assert k.numel() == 3
    k2, _ = t.select_for_save(1, f)  # delta scores were reset
    assert k2.numel() == 0
    kb, _ = t.select_for_save(0, f)
    assert kb.numel() == 5
    deleted = t.shrink(0.98, 0.8, 30, 0.1, 1.0)
    assert deleted == 5 and t.size() == 5


def test_auc_calculator_matches_sklearn():
    from sklearn.metrics import roc_auc_score

    torch.manual_seed(0)
    p = torch.rand(5000)
    y = (torch.rand(5000) < p).float()
    c = h.AucCalculator(1000000)
    c.add(p, y)
    c.compute()
    assert c.auc == pytest.approx(roc_auc_score(y.numpy(), p.numpy()), abs=1e-4)
    assert c.actual_ctr == pytest.approx(float(y.mean()))
    assert c.predicted_ctr == pytest.approx(float(p.mean()), rel=1e-5)
    assert c.mae == pytest.approx(float((p - y).abs().mean()), rel=1e-5)
    assert c.size == 5000
    # one class only -> -0.5
    c.reset()
    c.add(p[:10], torch.zeros(10))
    c.compute()
    assert c.auc == -0.5


def test_wuauc():
    c = h.AucCalculator(1000)
    pred = torch.tensor([0.9, 0.1, 0.8, 0.3, 0.5, 0.6])
    lab = torch.tensor([1.0, 0.0, 0.0, 1.0, 1.0, 1.0])
    uid = torch.tensor([1, 1, 2, 2, 3, 3])
    c.add_uid(pred, lab, uid)
    c.compute_wuauc()
    # user1 auc 1, user2 auc 0, user3 has no negatives (skipped)
    assert c.user_cnt == 2
    assert c.uauc == pytest.approx(0.5, abs=1e-6)


def _dataset(slots):
    d = h.SlotDataset()
    d.set_slots([h.SlotDesc(*s) for s in slots])
    return d


def test_slot_parser_and_batch():
    d = _dataset([("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1),
                  ("s2", "uint64", True, False, 1), ("dense", "float", True, True, 3),
                  ("unused", "uint64", False, False, 1)])
    lines = [
        "1 1 2 11 12 1 21 2 0.5 1.5 1 7",
        "1 0 1 13 2 0 22 3 1 2 3 1 8",  # s2 has a 0 feasign -> dropped
        "1 1 1 0 1 0 1 1.0 1 9",  # no sparse feasign at all -> dropped
    ]
    assert d.add_lines(lines) == 2
    assert d.size() == 2
    assert d.num_sparse_slots() == 2 and d.dense_width() == 4
    keys, lod, dense = d.build_batch(0, 2, False)
    assert keys.tolist() == [11, 12, 13, 21, 22]
    assert lod.tolist() == [0, 2, 3, 3, 4, 5]
    torch.testing.assert_close(dense, torch.tensor([[1.0, 0.5, 1.5, 0.0], [0.0, 1.0, 2.0, 3.0]]))
    assert sorted(d.collect_keys(True).tolist()) == [11, 12, 13, 21, 22]


def test_slot_parser_logkey_and_rank_offset():
    d = _dataset([("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1)])
    d.set_parse(_pc(logkey=True))
    sid = "%016x" % 77

    def lk(cmatch, rank):
        return "0" * 11 + "%03x" % cmatch + "%02x" % rank + sid

    lines = [f"1 {lk(222, 1)} 1 1 1 5", f"1 {lk(223, 2)} 1 0 1 6", f"1 {lk(100, 1)} 1 0 1 7"]
    assert d.add_lines(lines) == 3
    assert d.search_ids().tolist() == [77, 77, 77]
    cr = d.cmatch_rank()
    assert (cr >> 32).tolist() == [222, 223, 100]
    off = d.merge_by_search_id()
    assert off.tolist() == [0, 3]
    ro = d.build_rank_offset(0, 3, 3)
    # ins0 rank1: peers rank1 -> idx0, rank2 -> idx1
    assert ro[0].tolist() == [1, 1, 0, 2, 1, -1, -1]
    assert ro[1].tolist() == [2, 1, 0, 2, 1, -1, -1]
    assert ro[2].tolist() == [-1, -1, -1, -1, -1, -1, -1]


def _pc(ins_id=False, logkey=False):
    pc = h.ParseConfig()
    pc.parse_ins_id = ins_id
    pc.parse_logkey = logkey
    return pc


def test_file_load_pipe_and_archive(tmp_path):
    d = _dataset([("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1)])
    d.set_parse(_pc(ins_id=True))
    files = []
    for i in range(3):
        p = tmp_path / f"part-{i}.txt"
        p.write_text("".join(f"1 ins{i}_{j} 1 {j % 2} 2 {100 + j} {200 + i}\n" for j in range(50)))
        files.append(str(p))
    d.set_filelist(files)
    d.set_thread_num(3)
    assert d.load_into_memory() == 150
    arch = str(tmp_path / "a.bin")
    d.save_archive(arch)
    d2 = _dataset([("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1)])
    assert d2.load_archive(arch, False) == 150
    k1, l1, x1 = d.build_batch(0, 150, False)
    k2, l2, x2 = d2.build_batch(0, 150, False)
    assert torch.equal(k1, k2) and torch.equal(l1, l2) and torch.equal(x1, x2)
    # pipe command path
    d3 = _dataset([("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1)])
    d3.set_parse(_pc(ins_id=True))
    d3.set_filelist(files[:1])
    d3.set_pipe_command("cat")
    assert d3.load_into_memory() == 50
    d4 = _dataset([("label", "uint64", True, True, 1), ("s1", "uint64", True, False, 1)])
    d4.set_parse(_pc(ins_id=True))
    d4.set_filelist(files[:1])
    d4.set_pipe_command("head -n 10")
    assert d4.load_into_memory() == 10


def test_flags_registry_env_override(monkeypatch):
    from paddlebox_amd.utils import flags

    flags.set_flags({"FLAGS_check_nan_inf": True})
    assert flags.get_bool("check_nan_inf")
    flags.set_flags({"check_nan_inf": False})
    assert not flags.get_bool("check_nan_inf")
    with pytest.raises(KeyError):
        flags.set_flags({"no_such_flag": 1})


def test_key_agent_dedups_and_loader_registers_keys(tmp_path):
    """Feed-pass key registration by the loader threads (KeyAgent) equals a
    walk over the loaded store (reference: AddKeys from data_set.cc merge
    threads into the PSAgent)."""
    import numpy as np

    from paddlebox_amd import _native

    ka = _native.host().KeyAgent(8)
    ka.add(torch.tensor([5, 7, 5, 0, -1, 9, 7], dtype=torch.int64))
    assert sorted(ka.keys().tolist()) == [5, 7, 9] and ka.size() == 3
    big = torch.randint(1, 1 << 62, (200000,), dtype=torch.int64)
    ka.add(big)
    ka.add(big[:5000])
    assert ka.size() == 3 + int(torch.unique(big).numel())

    import paddlebox_amd.fluid as fluid
    from paddlebox_amd.ps.box_wrapper import BoxWrapper
    from tests.test_fluid import S, _build, _files

    box = fluid.core.BoxWrapper(8, device="cpu", new=True)
    try:
        box.initialize_gpu_and_load_model(slot_vector=list(range(S)), max_keys=200000)
        seen = {}
        orig = box.end_feed_pass

        def spy(agent=None):
            seen["keys"] = agent.keys().clone()
            seen["native"] = agent.native.size()
            return orig(agent)

        box.end_feed_pass = spy
        main, startup, slots, label, dense, pred, loss = _build()
        ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
        ds.set_use_var([label] + slots + [dense])
        ds.set_batch_size(32)
        ds.set_thread(3)
        ds.set_filelist(_files(tmp_path, 3, 200))
        boxps = fluid.core.BoxPS(ds)
        boxps.read_ins_into_memory()
        want = np.unique(ds.collect_keys().numpy())
        got = np.unique(seen["keys"].numpy())
        assert seen["native"] == got.size > 0
        np.testing.assert_array_equal(got, want)
        h, _ = box.engine.table.export(True)
        assert h.numel() == want.size
    finally:
        BoxWrapper._instance = None


def test_pcoc_q_values_follow_records(tmp_path):
    """PCOC q values (pack_qvalue / store_qvalue, data_feed.cc:4945-4984):
    store_q_value writes one float per instance into the records' extension
    floats; a later batch over the same records (after a reshuffle, an archive
    round trip) carries them in its packed q tensor."""
    import paddlebox_amd.fluid as fluid
    from paddlebox_amd.data.dataset import PadBoxSlotDataset
    from paddlebox_amd.fluid.kernels import KERNELS

    ds = PadBoxSlotDataset(rank=0, world=1)
    ds._native.set_slots([h.SlotDesc("label", "uint64", True, True, 1), h.SlotDesc("s", "uint64", True, False, 1)])
    ds._configured = True
    n = 50
    ds.add_lines([f"1 {i % 2} 1 {1000 + i}" for i in range(n)])
    b = ds.build_batch(0, n)
    assert b.extra["q_values"].shape == (n, 2) and float(b.extra["q_values"].abs().sum()) == 0.0
    # store_q_value over this batch: q0 = key-derived, q1 = 2 * q0
    q0 = (b.keys.float() - 1000.0) / 10.0
    prog = fluid.Program()
    with fluid.program_guard(prog):
        a = fluid.layers.data(name="qa", shape=[1], dtype="float32")
        c = fluid.layers.data(name="qb", shape=[1], dtype="float32")
        fluid.layers._store_q_value([a, c])
    op = prog.global_block().ops[-1]

    class Ctx:
        batch = b
        env = {"qa": q0.view(-1, 1), "qb": (2 * q0).view(-1, 1)}

        def get(self, v):
            return self.env[v if isinstance(v, str) else v.name]

    KERNELS["store_q_value"](Ctx(), op)
    ds.local_shuffle(5)
    b2 = ds.build_batch(0, n)
    want = (b2.keys.float() - 1000.0) / 10.0
    torch.testing.assert_close(b2.extra["q_values"][:, 0], want)
    torch.testing.assert_close(b2.extra["q_values"][:, 1], 2 * want)
    # archive keeps them
    ds._native.save_archive(str(tmp_path / "arch"))
    ds2 = PadBoxSlotDataset(rank=0, world=1)
    ds2._native.set_slots([h.SlotDesc("label", "uint64", True, True, 1), h.SlotDesc("s", "uint64", True, False, 1)])
    ds2._configured = True
    ds2._native.load_archive(str(tmp_path / "arch"), False)
    b3 = ds2.build_batch(0, n)
    torch.testing.assert_close(b3.extra["q_values"][:, 0], (b3.keys.float() - 1000.0) / 10.0)


def test_dump_debug_flags(tmp_path):
    """FLAGS_padbox_dump_debug_lineid (only the matching line is dumped) and
    FLAGS_dump_filed_same_as_aibox (field header = name before '.', no ':len'),
    boxps_worker.cc:1777-1815."""
    from paddlebox_amd.utils.flags import set_flags

    ids = [f"{i:032d}" for i in range(4)]
    mat = torch.arange(8, dtype=torch.float32).view(4, 2)

    def run(sub, flags):
        set_flags(flags)
        try:
            w = h.DumpWriter(str(tmp_path / sub), 0, 1)
            w.dump_fields(ids, ["fc.tmp_0"], [mat], 0, 1, False)
            w.flush()
        finally:
            set_flags({"FLAGS_padbox_dump_debug_lineid": "", "FLAGS_dump_filed_same_as_aibox": False})
        out = []
        for f in sorted((tmp_path / sub).rglob("*")):
            if f.is_file():
                out += [ln for ln in f.read_text().splitlines() if ln]
        return out

    plain = run("a", {})
    v = lambda x: f"{x:.9f}"  # noqa: E731  (the writer's float format)
    assert len(plain) == 4 and plain[1] == f"{ids[1]}\tfc.tmp_0:2:{v(2)}:{v(3)}"
    one = run("b", {"FLAGS_padbox_dump_debug_lineid": ids[2]})
    assert one == [f"{ids[2]}\tfc.tmp_0:2:{v(4)}:{v(5)}"]
    ai = run("c", {"FLAGS_dump_filed_same_as_aibox": True})
    assert ai[0] == f"{ids[0]}\tfc:0:{v(1)}"


def test_init_afs_api_configures_the_file_client(tmp_path):
    """init_afs_api ignored its arguments.  It now configures the
    process-wide native client (reference InitAfsAPI, box_wrapper.h:721-734:
    fs_ugi = "user,passwd") that model IO and the pass loaders use."""
    from paddlebox_amd.ps.box_wrapper import BoxWrapper

    box = BoxWrapper(8, device="cpu")
    try:
        fake = tmp_path / "hadoop"
        fake.write_text("#!/bin/sh\necho \"$@\" >> " + str(tmp_path / "calls.txt") + "\n")
        fake.chmod(0o755)
        assert box.init_afs_api("afs://nn.example:9000", "alice", "s3cret", "/etc/hadoop",
                                hadoop_bin=str(fake)) == 0
        assert box.use_afs_api
        pre = box.fs._m.remote_prefix()
        assert "fs.default.name=" in pre and "afs://nn.example:9000" in pre
        assert "hadoop.job.ugi=" in pre and "alice,s3cret" in pre
        assert "--config" in pre and "/etc/hadoop" in pre
        box.fs.makedir("afs://nn.example:9000/user/alice/model")
        calls = (tmp_path / "calls.txt").read_text()
        assert "-mkdir" in calls and "alice,s3cret" in calls and "/user/alice/model" in calls
    finally:
        box.fs.destory()
        BoxWrapper._instance = None
