"""Adam state at the checkpoint boundary uses the reference's conventions
(ADVICE r2): fluid's AdamOptimizer initialises <param>_beta{1,2}_pow_acc_0 to
beta and multiplies after each update (python/paddle/fluid/optimizer.py
AdamOptimizer._create_accumulators / _append_optimize_op), so after t updates
the accumulator holds beta^(t+1); FlatAdam keeps beta^t.  A reference-style
fresh accumulator (= beta) must load as "no step taken yet"."""
import numpy as np
import pytest
import torch

import paddlebox_amd.fluid as fluid
from paddlebox_amd.ps.box_wrapper import BoxWrapper
from tests.test_fluid import S, _build, _files


@pytest.fixture
def box():
    BoxWrapper._instance = None
    b = fluid.core.BoxWrapper(8, device="cpu", new=True)
    b.cfg.sgd.mf_create_thresholds = 0.0
    b.initialize_gpu_and_load_model(slot_vector=list(range(S)), max_keys=200000)
    yield b
    BoxWrapper._instance = None


def _session(box, tmp_path):
    scope = fluid.Scope()
    main, startup, slots, label, dense, pred, loss = _build()
    exe = fluid.Executor(fluid.CPUPlace())
    exe.run(startup, scope=scope)
    ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
    ds.set_use_var([label] + slots + [dense])
    ds.set_batch_size(64)
    ds.set_filelist(_files(tmp_path, 1, 200))
    ds.disable_shuffle()
    boxps = fluid.core.BoxPS(ds)
    boxps.read_ins_into_memory()
    boxps.begin_pass()
    exe.train_from_dataset(main, ds, scope=scope, fetch_list=[loss], print_period=1000)
    boxps.end_pass()
    return exe.sessions_for(main)[0]


def test_beta_pow_accumulators_follow_reference_convention(box, tmp_path):
    s = _session(box, tmp_path)
    opt = s.opts[0]
    steps = round(float(np.log(float(opt.pows[0])) / np.log(opt.b1)))
    assert steps == 4  # 200 records / batch 64
    st = s.optimizer_state()
    acc1 = [k for k in st if k.endswith("_beta1_pow_acc_0")]
    assert acc1
    for k in acc1:
        assert float(st[k]) == pytest.approx(opt.b1 ** (steps + 1), rel=1e-6)
    for k in (k for k in st if k.endswith("_beta2_pow_acc_0")):
        assert float(st[k]) == pytest.approx(opt.b2 ** (steps + 1), rel=1e-6)
    # a fresh reference accumulator (value = beta, zero moments) = no update taken
    fresh = {}
    for k, v in st.items():
        if k.endswith("_beta1_pow_acc_0"):
            fresh[k] = np.array([opt.b1], dtype=np.float32)
        elif k.endswith("_beta2_pow_acc_0"):
            fresh[k] = np.array([opt.b2], dtype=np.float32)
        else:
            fresh[k] = np.zeros(tuple(v.shape), dtype=np.float32)
    assert s.load_optimizer_state(fresh) > 0
    torch.testing.assert_close(opt.pows, torch.ones(2))
    assert float(opt.m.abs().sum()) == 0.0
    # round trip of the state just exported restores the powers exactly
    s.load_optimizer_state({k: np.asarray(v) for k, v in st.items()})
    assert float(opt.pows[0]) == pytest.approx(opt.b1 ** steps, rel=1e-6)


def test_optimizer_file_records_pow_convention(box, tmp_path):
    """save_persistables marks its optimizer file with the beta-pow convention;
    a file without the marker (written before it existed) holds raw beta^t
    powers and loads without the beta^(t+1) conversion."""
    from safetensors import safe_open
    from safetensors.numpy import save_file

    from paddlebox_amd.fluid import io as fio

    s = _session(box, tmp_path)
    opt = s.opts[0]
    pows = opt.pows.clone()
    d = tmp_path / "ckpt"
    d.mkdir()
    st = {k: np.ascontiguousarray(np.asarray(v)) for k, v in s.optimizer_state().items()}
    save_file(st, str(d / "marked.safetensors"), metadata={"beta_pow_convention": "reference"})
    with safe_open(str(d / "marked.safetensors"), "np") as f:
        assert f.metadata()["beta_pow_convention"] == "reference"
    # legacy layout: the raw powers under the same names, no marker
    legacy = dict(st)
    for k in legacy:
        if k.endswith("_beta1_pow_acc_0"):
            legacy[k] = pows[0:1].numpy().copy()
        elif k.endswith("_beta2_pow_acc_0"):
            legacy[k] = pows[1:2].numpy().copy()
    opt.pows.fill_(0.5)
    s.load_optimizer_state(legacy, reference_pows=False)
    torch.testing.assert_close(opt.pows, pows)
    opt.pows.fill_(0.5)
    s.load_optimizer_state(st, reference_pows=True)
    torch.testing.assert_close(opt.pows, pows)
    assert fio._OPT_FILE.endswith(".safetensors")
