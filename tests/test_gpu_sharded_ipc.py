"""The GPU sharded sparse step across PROCESSES (the multi-process
test only covered the CPU branch).  W ranks run on the one GPU of the test box,
each its own process with its own table shard, and exchange keys / values /
gradients over the IPC mesh (csrc/hip/ipc.hip: the same peer-write kernels
that run over xGMI on an 8-GPU node).  Checked against one unsharded CPU
engine processing the union batch, like test_sharded_loopback.py.  A second
test runs bench.py's whole graph-captured DeepFM step with W ranks on the
one GPU (--same-gpu: IPC meshes for the sparse exchange and the dense
all-reduce, gloo control plane)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batches(W, B, S, steps):
    from paddlebox_amd.data.synthetic import ragged_batch

    return [[ragged_batch(B, S, 4, 60, seed=100 * step + r, device="cpu") for r in range(W)] for step in range(steps)]


def _cfg():
    from paddlebox_amd.ps.config import PSConfig

    cfg = PSConfig(embedx_dim=8)
    cfg.sgd.mf_create_thresholds = 0.0
    return cfg


def _worker(rank, W, port, B, S, steps, q):
    try:
        import torch.distributed as dist

        from paddlebox_amd.ops import reference as ref
        from paddlebox_amd.parallel.comm import TorchDistComm
        from paddlebox_amd.ps.sparse_engine import SeqpoolParams, SparseEngine

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=W)
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        batches = _batches(W, B, S, steps)
        torch.manual_seed(0)
        douts = [[torch.randn(B, S * 11) * 0.01 for _ in range(W)] for _ in range(steps)]
        eng = SparseEngine(_cfg(), max_keys=4096, device=dev, capacity=10000, comm=TorchDistComm(),
                           exchange_capacity=2048, exchange="ipc")
        assert eng.exchange_mode == "ipc", eng.exchange_mode
        sp = SeqpoolParams()
        outs = []
        for step in range(steps):
            # feed pass of the union key set: every rank inserts the keys it owns
            allk = torch.cat([b.keys for b in batches[step]])
            h = torch.unique(ref.mix64(allk[allk != -1]))
            eng.insert_local_mixed(h[ref.owner_of(h, W) == rank].to(dev), init_embedx=True)
            b = batches[step][rank]
            out = torch.zeros(B, S * 11, device=dev)
            st = eng.pull_seqpool_cvm(b.keys.to(dev), b.lod.to(dev), B, S, out, 0, sp)
            outs.append(out.cpu())
            eng.push_seqpool_cvm(st, douts[step][rank].to(dev), b.cvm.to(dev), 0, sp, float(B))
        torch.cuda.synchronize()
        ovf = eng.check_overflow()
        hk, v = eng.table.export(True)
        dist.barrier()
        q.put((rank, outs, hk.cpu(), v.cpu(), ovf))
        for m in eng.xmesh:
            m.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), None, None, None))


@pytest.mark.parametrize("W,mode", [(2, "unfused"), (4, "unfused"), (2, "fused"), (4, "fused")])
def test_sharded_gpu_step_multiprocess_ipc(W, mode, monkeypatch):
    """mode: fused = the owner pack inside the key exchange and the owner
    probe + gather inside the answer exchange (k_ipc_pack_exchange /
    k_ipc_answer_exchange, PBX_PACK_EXCHANGE=1); unfused = pack, exchange,
    probe + gather, exchange as four launches (the default)."""
    monkeypatch.setenv("PBX_PACK_EXCHANGE", "1" if mode == "fused" else "0")
    from paddlebox_amd.ops import reference as ref
    from paddlebox_amd.ps.sparse_engine import SeqpoolParams, SparseEngine
    from tests.test_sharded_loopback import concat_batches

    B, S, steps = 24, 4, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, W, port, B, S, steps, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(W):
        r, outs, hk, v, ovf = q.get(timeout=240)
        res[r] = (outs, hk, v, ovf)
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    for r in range(W):
        assert not isinstance(res[r][0], str), res[r][0]
        assert res[r][3] is False, f"rank {r}: exchange overflow"
    # oracle: one CPU engine, union batch
    batches = _batches(W, B, S, steps)
    torch.manual_seed(0)
    douts = [[torch.randn(B, S * 11) * 0.01 for _ in range(W)] for _ in range(steps)]
    eng = SparseEngine(_cfg(), max_keys=4096 * W, device=torch.device("cpu"), capacity=10000 * W)
    sp = SeqpoolParams()
    for step in range(steps):
        ub = concat_batches(batches[step])
        eng.register_keys(ub.keys, init_embedx=True)
        out = torch.zeros(ub.B, S * 11)
        st = eng.pull_seqpool_cvm(ub.keys, ub.lod, ub.B, S, out, 0, sp)
        for r in range(W):
            torch.testing.assert_close(res[r][0][step], out[r * B:(r + 1) * B], rtol=1e-4, atol=1e-5)
        eng.push_seqpool_cvm(st, torch.cat(douts[step]), ub.cvm, 0, sp, float(B))
    allh = torch.cat([res[r][1] for r in range(W)])
    allv = torch.cat([res[r][2] for r in range(W)])
    assert allh.numel() == torch.unique(allh).numel() == eng.table.size()
    for r in range(W):
        assert bool((ref.owner_of(res[r][1], W) == r).all())
    exp = eng.table.read(allh)
    torch.testing.assert_close(allv[:, :14], exp[:, :14], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("W", [2, 4])
def test_bench_step_same_gpu_ranks(W):
    """bench.py's captured N-rank DeepFM step (IPC sparse exchange + IPC dense
    all-reduce, data_norm stats in the gradient bucket), W ranks on one GPU."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(W), "--same-gpu", "--steps", "10", "--warmup", "3", "--total-features", "4e6",
           "--batch-per-gpu", "2048", "--num-batches", "8", "--graph-warm", "4"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    c = out["config"]
    assert out["n_gpus"] == W and c["ranks_seen"] == W
    assert c["sparse_exchange"] == "ipc" and c["dense_allreduce"] == "ipc" and c["same_gpu_rehearsal"]
    assert out["value"] > 0
    assert "loss=nan" not in p.stderr
