"""CTR dense tower: fused head (data_norm + first-order/FM) + MLP + loss as
one autograd node, on the three-launch HIP tower (csrc/hip/tower.hip).

Forward  : k_head_fwd (data_norm -> MLP input (bf16, or fp32 for the fp32 tower)
           in row-major and m-packed layouts, lin = first-order + FM,
           data_norm batch-stat partials)
           k_tower_fwd (all ReLU layers, output GEMV, sigmoid, log-loss,
           d loss/d logit, AUC histogram)
Backward : k_tower_bwd (dX chain) + k_tower_dw (grouped dW GEMM, bias /
           output-layer grads, data_norm stats) + k_head_bwd (dx for the
           sparse push)

The extra logit term is either the head's ``lin`` (DeepFM: first + FM; Wide&Deep:
first-order "wide" part) or an external tensor (DCN-V2 cross branch), whose
gradient is ``dz * dloss``.

Reference semantics: data_norm (paddle/fluid/operators/data_norm_op.cu:38-104),
fc + relu, sigmoid + log_loss, auc (paddle/phi/kernels/gpu/auc_kernel.cu:25-80).
CPU tensors run the same math in plain fp32 PyTorch.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .. import _native
from ..parallel.comm import allreduce_sum, collective_active
from ..parallel.dense import add_grad_producer, join_grad_producers, pop_pre_head_event
from . import reference as ref
from .mlp import _ensure_grad


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


def _collectives_in_step() -> bool:
    """RCCL work in the step (multi-rank or a forced-collectives rehearsal):
    the dW side stream then only delays the dense all-reduce that overlaps
    the sparse exchange (measured 0.478 vs 0.389 ms/step on the 1-rank
    rehearsal), so the dW GEMM stays on the compute stream."""
    if os.environ.get("PBX_FORCE_COLLECTIVES") == "1":
        return True
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class _CtrTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, extra, label, t: "CtrTower", *params):
        h = _native.hip()
        mlp, dn = t.mlp, t.dn
        pre_head = pop_pre_head_event(t.uid) if x.is_cuda else None
        if pre_head is not None:
            # overlapped optimizer: the previous step's dW (which reads this
            # head's output buffers) and data_norm update are done; its Adam
            # may still run on the side stream -- joined below, before the
            # tower reads the weights
            torch.cuda.current_stream(x.device).wait_event(pre_head)
        elif x.is_cuda:
            join_grad_producers()  # a previous dW still reading the activations (no optimizer step between)
        B = x.shape[0]
        ws = mlp.tower_workspace(B, x.device, fp32=t.fp32, x3=t.x3)
        if pre_head is None:
            mlp.ensure_packed()
        x = x.contiguous()
        yt = t._cross_yt(B, x.device) if t.cross is not None else None
        Cp = ws.K0p  # MLP input width: padded to 32 (bf16 / x3 tower) / 16 (fp32 tower)
        # the x3 tower takes fp32 rows and m-packs their hi / lo halves itself
        ymp = None if t.x3 else ws.x0mp()
        if dn is not None:
            part = t._dn_part(B, x.device)
            _, lin, means, scales = h.head_fwd(x, t.S, t.Eo, t.ew_col, t.D, Cp, dn.batch_size,
                                               dn.batch_sum, dn.batch_square_sum, y_out=ws.x0(), yT_out=yt,
                                               ymp_out=ymp, stat_part=part)
        else:
            _, lin, means, scales = h.head_fwd(x, t.S, t.Eo, t.ew_col, t.D, Cp, None, None, None,
                                               y_out=ws.x0(), yT_out=yt, ymp_out=ymp)
        if extra is not None:
            lin_use = extra.detach().contiguous().float().view(-1)
        elif t.use_head_lin:
            lin_use = lin
        else:
            lin_use = None
        if t.cross is not None:
            # DCN-V2 cross stack on the normalised input the head just wrote
            # (x0 and its transposed copy): its logit joins the tower's loss.
            # Its weights are updated by the overlapped Adam too: join it first
            # (the cross forward read net.w / w_c under the update)
            if pre_head is not None:
                join_grad_producers()
            net, w_c = t.cross
            xw = net.workspace(ws.x0())
            s = xw.forward(ws.x0(), [w.detach() for w in net.w], [b.detach() for b in net.b], w_c.detach())
            lin_use = s if lin_use is None else lin_use + s
            ctx.yt = yt
        if pre_head is not None:
            join_grad_producers()
            mlp.ensure_packed()
        auc = t.auc
        # a [B] / [B, 1] label may be a strided column view (read in place)
        lab = label if label.dtype == torch.float32 and label.dim() in (1, 2) else label.float().contiguous().view(-1)
        loss, pred, dz = ws.forward(list(mlp.b), mlp.w_out.view(-1), mlp.b_out, lin_use, lab,
                                    auc[0] if auc else None, auc[1] if auc else None, auc[2] if auc else None)
        ctx.t, ctx.ws = t, ws
        ctx.save_for_backward(x)
        ctx.means, ctx.scales, ctx.dz = means, scales, dz
        ctx.has_extra = extra is not None
        ctx.mark_non_differentiable(pred)
        # no zero-filled grad for pred, no ones-filled grad needed for the loss
        # (a None dloss means 1): two fill launches less per step
        ctx.set_materialize_grads(False)
        return loss.view(()), pred

    @staticmethod
    def backward(ctx, gl, gp):
        h = _native.hip()
        t, ws = ctx.t, ctx.ws
        mlp, dn = t.mlp, t.dn
        (x,) = ctx.saved_tensors
        B = x.shape[0]
        mlp.ensure_grads()
        if gl is not None:
            gl = gl.contiguous().float().view(1)
        dn_on = dn is not None and dn.training and dn.update_norm
        args = (gl, mlp.w_out.detach().view(-1), [w.grad for w in mlp.w], [b.grad for b in mlp.b],
                mlp.w_out.grad.view(-1), mlp.b_out.grad, True, t._dn_part(B, x.device) if dn_on else None,
                h.head_blocks(B) if dn_on else 0, dn.eps if dn is not None else 0.0, dn.stats if dn_on else None)

        # with a DCN-V2 cross stack the dense gradients are final only after
        # the cross backward below: a dense tail that runs before it (dW
        # launched right after the dX chain, or no dW overlap) must not yet
        # fire on_dense_grads (the all-reduce / overlapped Adam would read the
        # cross weights' gradients unfinished)
        hook = {"after_cross": False}
        # single-process statistics: the dW launch's reduction workgroups also
        # fold them into the summaries (one k_dn_update launch less on the
        # side stream, ahead of the next step's head forward)
        dn_inline = (dn_on and not dn.fused_update and not getattr(dn, "update_in_hook", False)
                     and not getattr(dn, "stats_in_grad_bucket", False)
                     and not (dn.sync_stats and dn.group is not None and collective_active(dn.group))
                     and os.environ.get("PBX_DN_INLINE_UPDATE", "1") == "1")
        dnk = ({"dn_bsize": dn.batch_size, "dn_bsum": dn.batch_sum, "dn_bsq": dn.batch_square_sum,
                "dn_decay": float(dn.decay)} if dn_inline else {})

        # PBX_X3_FUSED_HEAD=1 (x3 tower, no cross stack): the head backward
        # inside the dX chain's last epilogue (k_tx3_bwd), one launch less --
        # measured slower (0.2611-0.2629 vs 0.2484-0.2487 ms/step with the
        # separate k_head_bwd, profiles/r6_x3_fused_head_ab.txt: the pass runs
        # at one 512-thread workgroup per CU behind the chain's LDS tiles,
        # where k_head_bwd spreads 1024 small workgroups), so off by default
        use_lin = t.use_head_lin and not ctx.has_extra
        fuse_head = (ws.x3 and t.cross is None and os.environ.get("PBX_X3_FUSED_HEAD", "0") == "1"
                     and x.dim() == 2 and x.dtype == torch.float32 and x.is_contiguous())
        hk = ({"head_x": x, "head_scales": ctx.scales, "hS": t.S, "hEo": t.Eo, "hew": t.ew_col, "hD": t.D,
               "hlin": bool(use_lin)} if fuse_head else {})

        def bwd(parts=3):
            return ws.backward(*args, parts=parts, **dnk, **(hk if parts & 1 else {}))

        def dense_tail():
            if dn_on and not getattr(dn, "stats_in_grad_bucket", False):
                if dn.sync_stats and dn.group is not None and collective_active(dn.group):
                    allreduce_sum(dn.stats, dn.group)  # the group's IPC mesh when registered
            if dn_on and not dn_inline and not dn.fused_update and not getattr(dn, "update_in_hook", False):
                h.data_norm_update(dn.batch_size, dn.batch_sum, dn.batch_square_sum, dn.stats, dn.decay)
            if t.on_dense_grads is not None:  # e.g. start the dense all-reduce, overlapped with the sparse push
                if t.cross is not None and not hook["after_cross"]:
                    hook["pending"] = True
                else:
                    t.on_dense_grads()

        deferred_dw = None
        if t.overlap_dw and x.is_cuda and (t.overlap_dw_collectives or not _collectives_in_step()):
            # dX chain on the compute stream; the dW GEMMs + bias / data_norm
            # reductions (and whatever consumes the dense grads) on a side
            # stream, concurrent with the head backward and the sparse push;
            # the optimizer joins it (parallel.dense.join_grad_producers)
            cur = torch.cuda.current_stream(x.device)
            dx0 = bwd(1)
            deferred_dw = torch.cuda.Event()
            deferred_dw.record(cur)
            if t.on_dx_done is not None:  # e.g. the next batch's key dedup on a side stream
                t.on_dx_done(deferred_dw)
            if not t.dw_after_head:
                _launch_dw(t, bwd, dense_tail, x.device, deferred_dw)
                deferred_dw = None
        else:
            dx0 = bwd()
            dense_tail()
        if t.cross is not None:
            # cross backward (d logit = dz); its x0 gradient is added into the
            # tower's dX0 before the data_norm / head backward below
            net, w_c = t.cross
            fusedx = net._xw.fused_forward
            # the fused chain scales d logit by the loss grad itself (no
            # elementwise launch on the critical path)
            ds = ctx.dz if (gl is None or fusedx) else (ctx.dz * gl).contiguous()
            dsk = {"ds_scale": gl} if (gl is not None and fusedx) else {}
            cargs = (ws.x0(), ctx.yt, ds, [_ensure_grad(w) for w in net.w], [_ensure_grad(b) for b in net.b],
                     w_c.detach(), _ensure_grad(w_c))
            # the cross dW (grouped GEMM + db / dw_c reductions) only feeds the
            # optimizer: on the side stream after the cross dX chain, beside the
            # head backward and the sparse push (PBX_CROSS_DW_SIDE=0: inline)
            cross_side = (t.overlap_dw and x.is_cuda and fusedx
                          and (t.overlap_dw_collectives or not _collectives_in_step())
                          and os.environ.get("PBX_CROSS_DW_SIDE", "1") == "1")
            cross_late = None
            if cross_side:
                cur = torch.cuda.current_stream(x.device)
                net._xw.backward(*cargs, dy_out=dx0, parts=1, **dsk)
                chain = torch.cuda.Event()
                chain.record(cur)

                def cross_dw():
                    side = t._side_stream(x.device)
                    side.wait_event(chain)
                    with torch.cuda.stream(side):
                        net._xw.backward(*cargs, dy_out=dx0, parts=2, **dsk)
                        if hook.get("pending"):  # the dense tail ran: the cross grads are final here
                            t.on_dense_grads()
                    add_grad_producer(side)
                    hook["after_cross"] = True
                    hook["pending"] = False

                # PBX_CROSS_DW_AFTER_HEAD=1: enqueue the side-stream cross dW
                # after the head backward, so the head follows the cross dX
                # chain on the compute stream without a fork in between
                if os.environ.get("PBX_CROSS_DW_AFTER_HEAD", "0") == "1":
                    # a pending dense tail (the tower dW ran first) fires inside
                    # cross_dw on the side stream; a later tower dW's tail runs
                    # after it on the same stream
                    cross_late = cross_dw
                    if not hook.get("pending"):
                        hook["after_cross"] = True
                else:
                    cross_dw()
            else:
                net._xw.backward(*cargs, dy_out=dx0, **dsk)
                hook["after_cross"] = True
            if hook.get("pending") and cross_late is None:
                # the dense tail already ran (on the dW side stream, or inline):
                # fire the hook where it ran, once the cross gradients are final
                cur = torch.cuda.current_stream(x.device)
                if t._side is not None and t.overlap_dw and x.is_cuda and deferred_dw is None and \
                        (t.overlap_dw_collectives or not _collectives_in_step()):
                    done = torch.cuda.Event()
                    done.record(cur)
                    side = t._side_stream(x.device)
                    side.wait_event(done)
                    with torch.cuda.stream(side):
                        t.on_dense_grads()
                else:
                    t.on_dense_grads()
        if fuse_head:
            dx = dx0  # the fused epilogue's head gradient
        else:
            dx, _ = h.head_bwd(x, dx0, ctx.dz if use_lin else None, t.S, t.Eo, t.ew_col, t.D, ws.K0p,
                               ctx.means, ctx.scales, dn.eps if dn is not None else 0.0, dlin_scale=gl,
                               want_stats=False)
        if t.cross is not None and cross_late is not None:
            cross_late()
        if deferred_dw is not None:
            # issued after the head backward (and the cross backward): both
            # depend only on the dX chain, and a dW launch enqueued first
            # fills the CUs and starves the head's workgroups (fp32 tower:
            # head_bwd 13 -> 95 us beside k_t32_dw, profiles/r3_s2_dw_after_head.txt)
            _launch_dw(t, bwd, dense_tail, x.device, deferred_dw)
        if t.on_head_done is not None:  # e.g. the next batch's key dedup beside the sparse push
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(x.device))
            t.on_head_done(ev)
        d_extra = (ctx.dz * gl if gl is not None else ctx.dz.clone()) if ctx.has_extra else None
        return (dx, d_extra, None, None) + (None,) * (len(t._params))


def _launch_dw(t, bwd, dense_tail, device, after: "torch.cuda.Event"):
    """The tower's dW GEMM + reductions and the dense tail on its side stream,
    ordered after the dX chain (event ``after``) only."""
    side = t._side_stream(device)
    side.wait_event(after)
    with torch.cuda.stream(side):
        bwd(2)
        dense_tail()
    add_grad_producer(side)


class CtrTower:
    """Binds a FusedMLP (+ optional DataNorm) into the fused tower.

    S slot blocks of width Eo (embed_w at ew_col, D embedx after it) followed by
    dense columns make up the input x [B, C]."""

    _n = 0  # towers created (CtrTower.uid)

    def __init__(self, mlp, dn, S: int, Eo: int, ew_col: int, D: int, use_head_lin: bool = True, cross=None,
                 fp32: bool = False):
        """``cross``: optional (CrossNetV2, w_c) whose width is the tower's
        padded input width: a DCN-V2 cross logit computed inside the tower
        from its normalised input and added to the MLP logit.
        ``fp32``: run the exact-fp32 tower (tower32.hip) instead of the
        bf16-operand one (the reference's fp32 fc precision)."""
        if fp32 and cross is not None:
            raise ValueError("the fp32 tower does not carry the DCN-V2 cross stack")
        self.fp32 = bool(fp32)
        # x3: fp32-precision tower on bf16 MFMA (tower_x3.hip: hi / lo bf16
        # halves, 3 products per MFMA step); set by the model's precision
        self.x3 = False
        self.mlp, self.dn = mlp, dn
        self.cross = cross
        self._yt = None
        self.S, self.Eo, self.ew_col, self.D = S, Eo, ew_col, D
        self.use_head_lin = use_head_lin
        # key of the overlapped optimizer's pre-head event (parallel.dense):
        # unique per tower for the process, unlike id(), which a later
        # tower can reuse while an event of the old one is still registered
        CtrTower._n += 1
        self.uid = CtrTower._n
        self.auc = None  # (table [2, T] f64, stats [5] f64, mask or None): fused AUC accumulation
        # called in the backward once every dense gradient (and data_norm
        # statistic) of the tower is final, before the sparse push runs
        self.on_dense_grads = None
        # called with an event on the compute stream once the dX chain is
        # enqueued (the tower's big MFMA kernels are then behind it): work that
        # should overlap the dW / head backward / sparse push forks from it
        self.on_dx_done = None
        self.on_head_done = None
        # run the dW GEMM on a side stream, overlapped with the head backward
        # and the sparse push (PBX_TOWER_OVERLAP_DW=0 turns it off)
        self.overlap_dw = os.environ.get("PBX_TOWER_OVERLAP_DW", "1") != "0"
        # with collectives in the step the dW stays on the compute stream
        # (an RCCL all-reduce on a side stream delayed the sparse exchange) --
        # unless the owner sets this: its dense all-reduce is an IPC mesh
        # launched from the dW stream (CtrTrainStep)
        self.overlap_dw_collectives = False
        # ... enqueued after the head backward, or right after the dX chain.
        # Measured (profiles/r3_s2_dw_after_head.txt): after the head for
        # DeepFM (0.255 vs 0.278 ms/step); with a DCN-V2 cross stack too since
        # the cross dW moved to the side stream: the compute stream then runs
        # dX chain -> cross dX chain -> head with no fork between them
        # (0.306-0.308 vs 0.325-0.326 ms/step; the cross dW after the head as
        # well, PBX_CROSS_DW_AFTER_HEAD=1: 0.339, profiles/r6_dcn_enqueue_order.txt).
        # PBX_DW_AFTER_HEAD=1/0 forces either.
        env = os.environ.get("PBX_DW_AFTER_HEAD")
        self.dw_after_head = (env != "0") if env is not None else True
        self._side = None
        self._part = None
        self._params = list(mlp.parameters())
        if cross is not None:
            self._params += list(cross[0].parameters()) + [cross[1]]

    def _cross_yt(self, B, dev):
        """x0^T for the cross dW GEMM: [pad64(D+1), pad64(B)] bf16, the head
        writes rows < D, row D stays 1 (the bias row)."""
        D = self.cross[0].dim
        r, c = (D + 1 + 63) // 64 * 64, (B + 63) // 64 * 64
        if self._yt is None or tuple(self._yt.shape) != (r, c):
            self._yt = torch.zeros(r, c, dtype=torch.bfloat16, device=dev)
            self._yt[D, :B] = 1.0
        return self._yt

    def _side_stream(self, dev):
        if self._side is None:
            from ..runtime.streams import side_stream

            self._side = side_stream(dev, "tower_dw")
        return self._side

    def _dn_part(self, B, device):
        h = _native.hip()
        n = h.head_blocks(B) * 2 * self.dn.C
        if self._part is None or self._part.numel() != n:
            self._part = torch.zeros(n, device=device)
        return self._part

    def __call__(self, x: torch.Tensor, label: torch.Tensor, extra: Optional[torch.Tensor] = None
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
        """(mean log-loss, prediction) for x [B, C]."""
        if x.is_cuda:
            return _CtrTowerFn.apply(x, extra, label, self, *self._params)
        return self._cpu(x, label, extra)

    def _cpu(self, x, label, extra):
        from .ctr import ctr_head, logit_logloss

        Cp = self.mlp.in_dim
        y, lin = ctr_head(x, self.dn, self.S, self.Eo, self.ew_col, self.D, Cp)
        deep = self.mlp(y)
        other = extra if extra is not None else (lin if self.use_head_lin else None)
        if self.cross is not None:
            from ..models.dcn_v2 import cross_logit

            c = cross_logit(y, self.cross[0], self.cross[1])
            other = c if other is None else other + c
        loss, pred = logit_logloss(deep, other, label)
        if self.auc is not None:
            ref.auc_accumulate(pred.detach(), label.view(-1), self.auc[0], self.auc[1], self.auc[2])
        return loss, pred
