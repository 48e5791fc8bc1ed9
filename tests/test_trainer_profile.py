"""Trainer profile mode (reference TrainFilesWithProfiler,
boxps_worker.cc:1358-1482) and worker core binding
(boxps_trainer.cc:165-193)."""
import os

import paddlebox_amd.fluid as fluid
from paddlebox_amd.ps.box_wrapper import BoxWrapper
from paddlebox_amd.runtime.affinity import _parse_cpulist
from tests.test_fluid import S, _build, _files


def test_profile_mode_reports_every_op_and_grad_op(tmp_path):
    box = fluid.core.BoxWrapper(8, device="cpu", new=True)
    try:
        box.cfg.sgd.mf_create_thresholds = 0.0
        box.initialize_gpu_and_load_model(slot_vector=list(range(S)), max_keys=200000)
        main, startup, slots, label, dense, pred, loss = _build()
        exe = fluid.Executor(fluid.CPUPlace())
        scope = fluid.Scope()
        exe.run(startup, scope=scope)
        ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
        ds.set_use_var([label] + slots + [dense])
        ds.set_batch_size(64)
        ds.set_filelist(_files(tmp_path, 1, 200))
        ds.disable_shuffle()
        boxps = fluid.core.BoxPS(ds)
        boxps.read_ins_into_memory()
        boxps.begin_pass()
        st = exe.train_from_dataset(main, ds, scope=scope, debug=True, print_period=1000)
        boxps.end_pass()
        prof = st["op_profile"]
        nb = st["batches"]
        assert nb == 4
        assert prof["fc"]["calls"] == 3 * nb  # fc x2 hidden + output
        assert prof["__pull_seqpool_cvm"]["calls"] == nb or prof["pull_box_sparse"]["calls"] == nb
        assert prof["dense sync + optimizer"]["calls"] == nb
        assert any(k.endswith("_grad") for k in prof)  # grad ops timed through autograd hooks
        assert abs(sum(r["pct"] for r in prof.values()) - 100.0) < 0.5
    finally:
        BoxWrapper._instance = None


def test_cpulist_parser():
    assert _parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert _parse_cpulist("") == []
    assert set(os.sched_getaffinity(0))  # the binding intersects with this set


def test_dump_main_program_and_op_debug(tmp_path, monkeypatch, caplog):
    """FLAGS_enable_dump_main_program writes the lowered op list;
    FLAGS_padbox_enable_print_op_debug logs each op as it runs."""
    import numpy as np

    from paddlebox_amd.utils.flags import set_flags

    monkeypatch.chdir(tmp_path)
    set_flags({"FLAGS_enable_dump_main_program": True, "FLAGS_padbox_enable_print_op_debug": True})
    try:
        main, startup = fluid.Program(), fluid.Program()
        with fluid.program_guard(main, startup), fluid.unique_name.guard():
            x = fluid.layers.data("x", shape=[3], dtype="float32")
            y = fluid.layers.fc(x, 2, name="f")
            z = fluid.layers.reduce_sum(y)
        exe = fluid.Executor(fluid.CPUPlace())
        scope = fluid.Scope()
        exe.run(startup, scope=scope)
        with caplog.at_level("INFO", logger="pbx"):
            exe.run(main, feed={"x": np.ones((4, 3), np.float32)}, fetch_list=[z], scope=scope)
        text = (tmp_path / "device_0_ops_test.txt").read_text()
        assert "fc" in text and "reduce_sum" in text
        assert any("op fc" in r.getMessage() for r in caplog.records)
    finally:
        set_flags({"FLAGS_enable_dump_main_program": False, "FLAGS_padbox_enable_print_op_debug": False})
