"""The data-parallel CTR training step on one rank, as bench.py times it.

One object builds, over a shared :class:`~paddlebox_amd.ps.sparse_engine.SparseEngine`:

* the model (DeepFM or DCN-V2) at its MLP precision (exact fp32 or bf16 tower);
* the dense arena, one fused Adam launch (with the tower weight re-pack and the
  data_norm summary update folded in);
* on several ranks, the dense gradient all-reduce: the in-house IPC mesh
  (self-tested, one collective kernel, side stream, launched from the tower's
  dense-grads hook so it overlaps the sparse push) with RCCL as the fallback,
  and the data_norm batch statistics riding in the same all-reduce (tail of the
  gradient buffer);
* ``train_step(batch)``: forward, backward (sparse push with fused Adagrad
  inside the pull's backward), dense sync, Adam -- capturable into one HIP
  graph (runtime/graph_step.py).

Reference: the BoxPSWorker step, ``boxps_worker.cc:1191-1258`` (dense sync
modes) and ``:1296-1324`` (op loop); the dense sync hook
``box_wrapper.h:686-719``.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import torch
import torch.distributed as dist

from .. import _native

from ..parallel.dense import DenseArena, DenseSync, FlatAdam, join_grad_producer_upto_now, join_grad_producers


def make_ipc_mesh(nbytes: int, device, group=None, log=None):
    """A self-tested IPC mesh of ``nbytes`` per slot, or None (caller falls
    back to RCCL).  Collective over ``group``: every rank must call it."""
    from ..parallel.ipc import IpcMesh, IpcMeshError

    try:
        # dense collectives (gradient all-reduce, data_norm statistics,
        # c_allreduce_sum) queue on the dense-sync side stream, in issue order
        # (DenseSync.launch issues there itself: no fork on the hot path; a
        # fork from the tower's dW stream back into it, inside a captured
        # graph, crashed the capture)
        m = IpcMesh(nbytes, group=group, device=device, stream="dense_sync")
    except IpcMeshError as e:
        if log:
            log(f"IPC mesh unavailable ({e}); RCCL all-reduce")
        return None
    return m  # self-tested by its constructor (payload check, agreed over the group)


class CtrTrainStep:
    def __init__(self, engine, model_name: str = "deepfm", precision: str = "fp32", num_slots: int = 26,
                 dense_dim: int = 13, hidden: Sequence[int] = (400, 400, 400), cross_layers: int = 3,
                 multi: bool = False, dense: str = "ipc", same_gpu: bool = False, lr: float = 1e-3,
                 fused_auc: Optional[tuple] = None, log=None):
        """``multi``: data-parallel over the default process group (dense
        all-reduce + synced data_norm statistics).  ``dense``: "ipc" (the IPC
        mesh, RCCL fallback) or "rccl".  ``same_gpu``: every rank on one GPU
        (rehearsal): the IPC mesh is mandatory.  ``fused_auc``: (table, stats)
        accumulated by the tower's loss epilogue."""
        from ..models.dcn_v2 import DCNv2
        from ..models.deepfm import DeepFM

        device = engine.device
        self.device = device
        self.engine = engine
        dcn = model_name == "dcn_v2"
        fp32 = precision in ("fp32", "fp32x3")
        if dcn:
            if fp32:
                raise ValueError("DCN-V2 (BASELINE config 5) is a bf16-MLP config")
            model = DCNv2(engine, num_slots=num_slots, dense_dim=dense_dim, cross_layers=cross_layers,
                          hidden=tuple(hidden)).to(device)
        else:
            model = DeepFM(engine, num_slots=num_slots, dense_dim=dense_dim, hidden=tuple(hidden)).to(device)
        if fp32:
            model.set_precision(precision)
        self.model = model
        # the fused tower runs the whole dense side (bf16 operands, or exact fp32)
        self.fused = getattr(model, "use_tower", False) and (not fp32 or model.tower.fp32 or model.tower.x3)
        C = model.dn.C
        self.arena = DenseArena(model.parameters(), device, extra_grad=3 * C if multi and not dcn else 0)
        if multi:
            model.dn.group = dist.group.WORLD
            model.dn.sync_stats = True
            if self.fused and not dcn:
                # data_norm batch statistics are summed across ranks in the SAME
                # all-reduce as the dense gradients (tail of the gradient buffer)
                model.dn.stats = self.arena.grad_tail(3 * C)
                model.dn.stats_in_grad_bucket = True
        # one update launch for the dense side: Adam + tower weight re-pack +
        # data_norm summary update; grads zeroed by the same kernel
        self.opt = FlatAdam(self.arena, lr=lr, clear_grad=True)
        tower = getattr(model, "tower", None)
        # PBX_ADAM_OVERLAP (default on; one rank, fused tower): the update runs
        # on the dW side stream after the data_norm summary update, and the
        # NEXT step's head (data_norm + concat) starts once that summary update
        # is done -- only the tower forward waits for Adam (the step boundary
        # no longer serialises head_fwd behind the optimizer).  fp32 DeepFM
        # 0.3613 / 0.3610 -> 0.3559 / 0.3547 ms/step (profiles/r5_ab_finish_side_adam_overlap.txt);
        # DCN-V2 joins it before its cross forward (the cross weights are Adam's too)
        self.adam_overlap = (not multi and self.fused and tower is not None
                             and os.environ.get("PBX_ADAM_OVERLAP", "1") == "1")
        if self.fused:
            # the overlap keeps the data_norm update out of the Adam launch
            # (DCN-V2: the cross weights' bf16 copies are re-packed there too)
            self.opt.fuse(mlps=[model.mlp] + self._cross_of(model),
                          data_norms=[] if self.adam_overlap else [model.dn])
        self.ipc = None
        if multi and (dense == "ipc" or same_gpu):
            self.ipc = make_ipc_mesh(self.arena.grad.numel() * 4, device, log=log)
        if multi and same_gpu and (self.ipc is None or engine.exchange_mode != "ipc"):
            raise RuntimeError("same-GPU ranks need the IPC meshes (RCCL cannot run two ranks on one GPU)")
        # RCCL fallback: the gradient all-reduce stays on the default group and
        # runs in the step's order (no second communicator running concurrently
        # inside the captured graph: two RCCL communicators in flight on one
        # stream set can deadlock)
        self.sync = DenseSync(self.arena, mode="grad_allreduce", ipc=self.ipc)
        # PBX_ADAM_ON_SIDE=1 (one rank): the Adam update is issued from the
        # tower's dense-grads hook on the dW side stream (measured no faster)
        self.adam_side = ((not multi) and os.environ.get("PBX_ADAM_ON_SIDE", "0") == "1" and tower is not None
                          and not self.adam_overlap)
        self.adam_overlap_multi = False
        if self.adam_overlap:
            tower.on_dense_grads = self._side_update
        elif self.adam_side:
            tower.on_dense_grads = lambda: self.opt.step(1.0, join=False)
        elif tower is not None and (self.ipc is not None or not multi):
            # start the IPC all-reduce as soon as the tower's gradients are final
            tower.on_dense_grads = self.sync.launch
            # PBX_ADAM_OVERLAP_MULTI (default on; multi-rank, IPC dense mesh,
            # fused DeepFM tower): the Adam launch (with the data_norm update
            # fused in) follows the all-reduce on its own stream, so it runs
            # beside the sparse exchange chain instead of after it; the next
            # step's forward waits for it (pre-head event + grad-producer
            # join).  1-rank rehearsal 0.4227 / 0.4237 -> 0.4169 / 0.4192
            # ms/step (profiles/r5_adam_overlap_multi_ab.txt)
            if (multi and self.ipc is not None and self.fused and not dcn
                    and os.environ.get("PBX_ADAM_OVERLAP_MULTI", "1") == "1"):
                self.adam_overlap_multi = True
                tower.on_dense_grads = self._side_update_multi
                # the data_norm update leaves the Adam launch: the hook runs it
                # right after the all-reduce (which sums the statistics), and
                # the next step's head waits for it only, not for Adam
                self.opt.fuse(mlps=[model.mlp] + self._cross_of(model), data_norms=[])
                model.dn.fused_update = False
                model.dn.update_in_hook = True
            # multi-rank with the IPC dense mesh: the dW GEMM (and the all-reduce
            # it launches) may run on the side stream beside the head backward
            # and the sparse push exchange (PBX_OVERLAP_DW_IPC=1)
            tower.overlap_dw_collectives = (multi and self.ipc is not None
                                            and os.environ.get("PBX_OVERLAP_DW_IPC", "0") == "1")
        self.fused_auc = fused_auc is not None and self.fused
        if self.fused_auc:
            tower.auc = (fused_auc[0], fused_auc[1], None)
        self._auc = fused_auc
        self.one = torch.ones((), device=device)  # persistent d loss / d loss: no fill kernel per step
        # pipelined pull: the next batch (and its pull slot) to pool right
        # after this step's sparse push, under this step's dW GEMM
        self.next_batch = None
        self.next_slot = 0
        self._dedup_ev = None
        # the next batch's key dedup on its own side stream (PBX_SPLIT_PREFETCH):
        #   1: forked once this step's dX chain is enqueued -- it grabs the CUs
        #      ahead of the head backward and delays the dW start (0.413 vs
        #      0.398 ms/step, profiles/r4_pipeline_ab.txt);
        #   2: forked after the head backward, so it runs beside the sparse
        #      push and the dW GEMM (both wait on nothing it produces);
        # its pooling follows the push on this stream.  0 (default): the dedup
        # runs after the push on this stream.
        #   3: forked at the START of the step onto the tower's dW stream (idle
        #      until this step's dX chain is done), beside the head and tower
        #      forward / backward -- for the sharded step, whose dedup + exchange
        #      chain after the push is far longer than the dW GEMM
        # default 3 on several ranks: the sharded chain after the push (owner
        # update, sender hash dedup, two exchanges, owner gather) is far longer
        # than the dW GEMM -- 1-rank rehearsal 0.4221 / 0.4225 -> 0.3899 /
        # 0.3910 ms/step (mode 2: 0.449, profiles/r5_sharded_split3_ab.txt);
        # on one rank the dedup beside the tower measured slower (0.372 vs
        # 0.356, profiles/r5_split_prefetch_1rank_ab.txt)
        # DCN-V2 on one rank: 2 -- its latency-bound cross kernels leave room
        # for the dedup beside the push and the side-stream dW GEMMs (pipelined
        # front on: 0.3342 / 0.3341 vs 0.3513 / 0.3497 ms/step without the
        # pipeline, 0.374 / 0.353 with it and mode 0, 0.366 / 0.364 mode 3;
        # profiles/r6_dcn_split_ab.txt)
        mode = os.environ.get("PBX_SPLIT_PREFETCH", "3" if multi else ("2" if dcn else "0"))
        self.split_mode = mode if mode in ("1", "2", "3") else "0"
        self.split_prefetch = self.split_mode != "0" and tower is not None and hasattr(model, "prefetch_pool")
        if self.split_prefetch:
            if mode == "1":
                tower.on_dx_done = self._dedup_next
            elif mode == "2":
                tower.on_head_done = self._dedup_next

    @staticmethod
    def _cross_of(model):
        cross = getattr(model, "cross", None)
        return [cross] if cross is not None and hasattr(cross, "tower_workspaces") else []

    def _side_update(self):
        """On the dW side stream, after the data_norm summary update: mark the
        point the next step's head may start from, then Adam."""
        from ..parallel.dense import set_pre_head_event

        # PBX_HEAD_AFTER_ADAM=1: the mark after Adam instead -- the head then
        # waits for the update and the tower forward's own join of the side
        # stream is already satisfied (one cross-stream edge fewer on the
        # critical path when Adam ends before the pooling does)
        after = os.environ.get("PBX_HEAD_AFTER_ADAM", "0") == "1"
        if after:
            self.opt.step(1.0, join=False)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        set_pre_head_event(self.model.tower.uid, ev)
        if not after:
            self.opt.step(1.0, join=False)

    def _side_update_multi(self):
        """Tower dense-grads hook (multi-rank overlapped optimizer): the
        gradient + statistics all-reduce, then Adam (data_norm update fused)
        on the all-reduce's stream; the next forward joins that stream."""
        from ..parallel.dense import add_grad_producer, set_pre_head_event

        self.sync.launch()
        st = self.sync._stream
        dn = self.model.dn
        with torch.cuda.stream(st):
            if dn.training and dn.update_norm:  # the statistics just summed in the gradient tail
                _native.hip().data_norm_update(dn.batch_size, dn.batch_sum, dn.batch_square_sum, dn.stats, dn.decay)
            ev = torch.cuda.Event()
            ev.record(st)  # the next step's head may start here
            self.opt.step(self.sync.grad_scale(), join=False)
        self.sync._launched = False  # joined by the next forward, not by before_step
        set_pre_head_event(self.model.tower.uid, ev)
        add_grad_producer(st)

    def set_next(self, batch, slot: int = 0):
        """Batch to prefetch (pool) at the end of each train_step (None: off)."""
        self.next_batch, self.next_slot = batch, int(slot)

    def _dedup_next(self, after):
        nb = self.next_batch
        if nb is None or not self.engine.can_prefetch_pull():
            return
        from .streams import side_stream

        st = side_stream(self.device, "graph_prefetch")
        st.wait_event(after)
        with torch.cuda.stream(st):
            self.engine.prefetch_dedup(nb.keys, self.next_slot)
            ev = torch.cuda.Event()
            ev.record(st)
        self._dedup_ev = ev

    def prefetch(self, batch, slot: int) -> bool:
        pre = getattr(self.model, "prefetch", None)
        return bool(pre(batch, slot)) if pre is not None else False

    def __call__(self, b):
        return self.train_step(b)

    def _dedup_next_early(self):
        """Split mode 3: the next batch's key dedup on the tower's dW stream,
        issued before this step's forward (the stream is idle until the dX
        chain; the dW launch queues behind the dedup)."""
        nb = self.next_batch
        if nb is None or not self.engine.can_prefetch_pull():
            return
        cur = torch.cuda.current_stream(self.device)
        st = self.model.tower._side_stream(self.device)
        if self.adam_overlap_multi:
            # only the dW stream's work so far (the previous dW reads the
            # activations this forward rewrites): the overlapped Adam on the
            # all-reduce stream stays pending -- the head waits for its
            # pre-head event, the tower for its join
            join_grad_producer_upto_now(st)
        else:
            join_grad_producers()  # the forward's own join below then finds nothing to wait for
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            self.engine.prefetch_dedup(nb.keys, self.next_slot)
            ev = torch.cuda.Event()
            ev.record(st)
        self._dedup_ev = ev

    def train_step(self, b):
        from ..ops.ctr import auc_accumulate

        if self.split_prefetch and self.split_mode == "3":
            self._dedup_next_early()
        loss, pred = self.model(b)
        loss.backward(self.one)
        if self.next_batch is not None:
            # the sparse push is on this stream already: pool the next batch
            # now, beside the dW GEMM on the tower's side stream
            if self._dedup_ev is not None:
                torch.cuda.current_stream(self.device).wait_event(self._dedup_ev)
                self._dedup_ev = None
                self.model.prefetch_pool(self.next_batch, self.next_slot)
            else:
                self.prefetch(self.next_batch, self.next_slot)
        if self.adam_overlap or self.adam_overlap_multi:
            pass  # the side stream runs the update; the next forward joins it after its head
        elif self.adam_side:
            join_grad_producers()  # the side stream ran the update
        else:
            self.sync.before_step()
            self.opt.step(self.sync.grad_scale())
        if self._auc is not None and not self.fused_auc:
            auc_accumulate(pred, b.label, self._auc[0], self._auc[1])
        return loss.detach()

    def close(self):
        if self.ipc is not None:
            self.ipc.close()
            self.ipc = None
