"""Program lowering: op list -> executable steps, with PaddleBox fusions.

The reference runs every op of the program through the generic operator
interpreter (``BoxPSWorker::TrainFiles``, ``fw/boxps_worker.cc:1278-1357``);
here the program is pattern-matched once and the CTR hot chains are replaced
by the fused MI355X kernels:

1. ``pull_box_sparse -> fused_seqpool_cvm``  =>  ``__pull_seqpool_cvm``: one
   fused dedup/probe/gather/pool/CVM kernel chain writing straight into the
   concat buffer; its backward is the fused push-merge + sparse Adagrad
   (no per-occurrence pull records are materialised).
2. ``concat([seqpool outs..., dense...], axis=1)`` consuming those outputs
   is absorbed: the fused op writes the concat buffer and the per-slot
   outputs become column views of it.
4. (GPU) ``data_norm -> __fused_mlp -> sigmoid / log-loss / mean``  =>
   ``__ctr_tower`` (the fused CTR tower of the DeepFM bench, ops/tower.py).
3. (GPU) ``fc(relu) -> ... -> fc(relu) [-> fc(size=1)]`` chains  =>
   ``__fused_mlp``: at the reference fc precision (fp32, default) one
   library fp32 GEMM per layer with the gradients accumulated into the arena;
   with FLAGS_padbox_fc_precision=bf16, bf16 MFMA GEMMs with fused bias/ReLU
   epilogues, a GEMV logit head, ReLU-mask prologues and split-K dW/db in the
   backward.  The fc weights of a fused chain are stored ``[out, in]``
   (padded to 8) in the dense arena; the scope exposes the logical
   ``[in, out]`` view.

The tower (4) runs the exact-fp32 MFMA tower (csrc/hip/tower32.hip) at fp32
and the bf16-operand tower at bf16; at fp32 it is formed only when the fp32
tower's LDS budget takes the chain's widths (ops/mlp.py tower_fp32_fits),
otherwise the chain stays on the fp32 ``__fused_mlp``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .framework import Operator, Program, Variable
from .kernels import KERNELS


def pad8(n: int) -> int:
    return (n + 7) // 8 * 8


@dataclass
class StorageSpec:
    """How a parameter is stored in the dense arena."""

    kind: str  # "plain" | "t_pad" ([out_p, in_p] transposed) | "pad" (1-D padded)
    shape: Tuple[int, ...]  # storage shape
    logical: Tuple[int, ...]  # fluid shape


@dataclass
class Lowered:
    steps: List[Operator]
    storage: Dict[str, StorageSpec] = field(default_factory=dict)
    fusions: List[str] = field(default_factory=list)
    # ops a collective transpiler appended: run after backward on the @GRAD
    # values (op_role 1) / after the optimizer update on the parameters (2)
    backward_ops: List[Operator] = field(default_factory=list)
    optimize_ops: List[Operator] = field(default_factory=list)

    def describe(self) -> str:
        return "\n".join(f"{op.type}: {op.input_arg_names} -> {op.output_arg_names}" for op in self.steps)


def _consumers(ops: List[Operator]) -> Dict[str, List[int]]:
    c: Dict[str, List[int]] = {}
    for i, op in enumerate(ops):
        for n in op.input_arg_names:
            c.setdefault(n, []).append(i)
    return c


def _synthetic(block, type_, inputs, outputs, attrs) -> Operator:
    op = Operator.__new__(Operator)
    op.block, op.type = block, type_
    op.inputs = {k: list(v) for k, v in inputs.items()}
    op.outputs = {k: list(v) for k, v in outputs.items()}
    op.attrs = dict(attrs)
    return op


_SEQPOOL_FUSABLE = {"fused_seqpool_cvm"}


def _fuse_pull_seqpool(ops: List[Operator], fetch: set, engine_cvm_offset: int, notes: List[str]):
    cons = _consumers(ops)
    out = list(ops)
    removed = set()
    for i, op in enumerate(ops):
        if op.type != "pull_box_sparse":
            continue
        outs = op.outputs["Out"]
        users = {j for v in outs for j in cons.get(v.name, [])}
        if len(users) != 1 or any(v.name in fetch for v in outs):
            continue
        j = users.pop()
        f = ops[j]
        if f.type not in _SEQPOOL_FUSABLE or [v.name for v in f.inputs["X"]] != [v.name for v in outs]:
            continue
        a = f.attrs
        if a.get("embedx_concate_size", 1) != 1 or a.get("cvm_offset", 2) != engine_cvm_offset:
            continue
        if any(len(cons.get(v.name, [])) != 1 for v in outs):
            continue
        fused = _synthetic(op.block, "__pull_seqpool_cvm", {"Ids": op.inputs["Ids"], "CVM": f.inputs["CVM"]},
                           {"Out": f.outputs["Out"]}, dict(a, size=op.attrs.get("size")))
        # the fused op must run where the seqpool ran (its CVM input may be computed after the pull)
        out[j] = fused
        removed.add(i)
        notes.append(f"pull_box_sparse+fused_seqpool_cvm ({len(outs)} slots) -> __pull_seqpool_cvm")
    return [op for k, op in enumerate(out) if k not in removed]


def _absorb_concat(ops: List[Operator], notes: List[str]):
    produced_at: Dict[str, int] = {}
    for i, op in enumerate(ops):
        for n in op.output_arg_names:
            produced_at[n] = i
    cons = _consumers(ops)
    removed = set()
    for i, op in enumerate(ops):
        if op.type != "__pull_seqpool_cvm" or op.outputs.get("Concat"):
            continue
        names = [v.name for v in op.outputs["Out"]]
        for j in sorted({k for n in names for k in cons.get(n, [])}):
            c = ops[j]
            if c.type != "concat" or c.attrs.get("axis", 0) not in (1, -1):
                continue
            xs = c.inputs["X"]
            if [v.name for v in xs[:len(names)]] != names:
                continue
            rest = xs[len(names):]
            # tail inputs must be available before the fused op runs
            if any(produced_at.get(v.name, -1) >= i for v in rest):
                continue
            op.inputs["Dense"] = list(rest)
            op.outputs["Concat"] = c.outputs["Out"]
            removed.add(j)
            notes.append(f"concat of {len(names)} seqpool outputs (+{len(rest)} dense) absorbed")
            break
    return [op for k, op in enumerate(ops) if k not in removed]


def _fuse_cvm(ops: List[Operator], fetch: set, notes: List[str]):
    """``concat([fill_constant_batch_size_like(1.0, [-1, 1]), cast(label ->
    float32)], axis=1)`` -- the canonical program's show/click CVM input --
    => ``__cvm_show_click``: a persistent [B, 2] buffer whose show column is
    1 once and whose click column is copied from the label each step (one
    launch instead of a fill, a cast and a concat)."""
    produced_at: Dict[str, int] = {}
    for i, op in enumerate(ops):
        for n in op.output_arg_names:
            produced_at[n] = i
    cons = _consumers(ops)
    out = list(ops)
    removed = set()
    for k, op in enumerate(ops):
        if op.type != "concat" or op.attrs.get("axis", 0) not in (1, -1) or len(op.inputs["X"]) != 2:
            continue
        sn, cn = op.inputs["X"][0].name, op.inputs["X"][1].name
        i, j = produced_at.get(sn, -1), produced_at.get(cn, -1)
        if i < 0 or j < 0 or sn in fetch or cn in fetch:
            continue
        fo, co = ops[i], ops[j]
        if fo.type != "fill_constant_batch_size_like" or co.type != "cast":
            continue
        if float(fo.attrs.get("value", 0)) != 1.0 or list(fo.attrs.get("shape", [])) != [-1, 1] \
                or fo.attrs.get("dtype") not in ("float32", None) or co.attrs.get("out_dtype") != "float32":
            continue
        if len(cons.get(sn, [])) != 1:
            continue
        out[k] = _synthetic(op.block, "__cvm_show_click", {"Label": co.inputs["X"]}, {"Out": op.outputs["Out"]}, {})
        removed.add(i)
        if len(cons.get(cn, [])) == 1:
            removed.add(j)  # else the float label also feeds the loss: the cast stays
        notes.append("fill_constant(1) + cast(label) + concat -> __cvm_show_click")
    return [op for q, op in enumerate(out) if q not in removed]


def _fc_ok(op: Operator) -> bool:
    return (op.type == "fc" and op.attrs.get("in_num_col_dims", 1) == 1 and len(op.inputs["Input"]) == 1
            and bool(op.inputs.get("Bias")) and len(op.inputs["W"][0].shape) == 2)


def _fuse_mlp(ops: List[Operator], fetch: set, storage: Dict[str, StorageSpec], notes: List[str]):
    cons = _consumers(ops)
    used = set()
    out = list(ops)
    removed = set()
    for i, op in enumerate(ops):
        if i in used or not _fc_ok(op) or op.attrs.get("activation_type") != "relu":
            continue
        chain = [i]
        cur = op
        head = None
        while True:
            o = cur.outputs["Out"][0].name
            us = cons.get(o, [])
            if o in fetch or len(us) != 1:
                break
            nxt = ops[us[0]]
            if not _fc_ok(nxt) or nxt.inputs["Input"][0].name != o:
                break
            if nxt.attrs.get("activation_type") == "relu":
                chain.append(us[0])
                cur = nxt
                continue
            if nxt.attrs.get("activation_type", "") == "" and nxt.inputs["W"][0].shape[1] == 1:
                head = us[0]
            break
        ws = [ops[k].inputs["W"][0] for k in chain]
        bs = [ops[k].inputs["Bias"][0] for k in chain]
        for w, b in zip(ws, bs):
            K, N = w.shape
            storage[w.name] = StorageSpec("t_pad", (pad8(N), pad8(K)), (K, N))
            storage[b.name] = StorageSpec("pad", (pad8(N),), (N,))
        ins = {"X": ops[i].inputs["Input"], "W": ws, "B": bs}
        last = ops[chain[-1]]
        attrs = {"out_dim": last.inputs["W"][0].shape[1]}
        if head is not None:
            h = ops[head]
            wo, bo = h.inputs["W"][0], h.inputs["Bias"][0]
            H = wo.shape[0]
            storage[wo.name] = StorageSpec("t_pad", (1, pad8(H)), (H, 1))
            storage[bo.name] = StorageSpec("plain", (1,), (1,))
            ins["WOut"], ins["BOut"] = [wo], [bo]
            outv = h.outputs["Out"]
        else:
            outv = last.outputs["Out"]
        fused = _synthetic(op.block, "__fused_mlp", ins, {"Out": outv}, attrs)
        end = head if head is not None else chain[-1]
        out[end] = fused
        for k in chain:
            used.add(k)
            if k != end:
                removed.add(k)
        notes.append(f"fc chain of {len(chain)} relu layers{' + logit head' if head is not None else ''}"
                     " -> __fused_mlp")
    return [op for k, op in enumerate(out) if k not in removed]


def _fuse_tower(ops: List[Operator], fetch: set, notes: List[str], fp32: bool = True):
    """(GPU) data_norm -> __fused_mlp(+logit head) -> {sigmoid, sigmoid_cross_
    entropy_with_logits -> reduce_mean}  =>  ``__ctr_tower``: the fused CTR
    tower (csrc/hip/tower.hip: data_norm head, MFMA MLP with activations kept
    on chip, sigmoid + log-loss, one backward chain with the data_norm
    statistics)."""
    produced_at: Dict[str, int] = {}
    for i, op in enumerate(ops):
        for n in op.output_arg_names:
            produced_at[n] = i
    cons = _consumers(ops)
    out = list(ops)
    removed = set()
    for m, mop in enumerate(ops):
        if mop.type != "__fused_mlp" or not mop.inputs.get("WOut"):
            continue
        xn = mop.inputs["X"][0].name
        d = produced_at.get(xn, -1)
        if d < 0 or ops[d].type != "data_norm" or len(cons.get(xn, [])) != 1 or xn in fetch:
            continue
        dop = ops[d]
        if dop.inputs.get("scale_w") or dop.inputs.get("bias") or dop.attrs.get("slot_dim", -1) > 0:
            continue
        logit = mop.outputs["Out"][0].name
        users = cons.get(logit, [])
        if logit in fetch or len(users) != 2:
            continue
        types = {ops[u].type: u for u in users}
        if set(types) != {"sigmoid", "sigmoid_cross_entropy_with_logits"}:
            continue
        sg, xe = ops[types["sigmoid"]], ops[types["sigmoid_cross_entropy_with_logits"]]
        xen = xe.outputs["Out"][0].name
        xu = cons.get(xen, [])
        if xen in fetch or len(xu) != 1 or ops[xu[0]].type != "reduce_mean" or xe.attrs.get("normalize"):
            continue
        rm = ops[xu[0]]
        if rm.attrs.get("dim") not in (None, [], [0, 1], [-1, 0]) and not rm.attrs.get("reduce_all", True):
            continue
        lab = xe.inputs["Label"][0].name
        if produced_at.get(lab, -1) >= m:
            continue
        if fp32:
            from ..ops.mlp import tower_fp32_fits

            widths = [mop.inputs["W"][0].shape[0]] + [w.shape[1] for w in mop.inputs["W"]]
            if not tower_fp32_fits([pad8(w) for w in widths]):
                continue
        ins = {"X": dop.inputs["X"], "Label": xe.inputs["Label"], "W": mop.inputs["W"], "B": mop.inputs["B"],
               "WOut": mop.inputs["WOut"], "BOut": mop.inputs["BOut"],
               "BatchSize": dop.inputs["BatchSize"], "BatchSum": dop.inputs["BatchSum"],
               "BatchSquareSum": dop.inputs["BatchSquareSum"]}
        attrs = {k: dop.attrs.get(k) for k in ("epsilon", "summary_decay_rate", "sync_stats", "update_norm")}
        lp = produced_at.get(lab, -1)
        if lp >= 0 and ops[lp].type == "cast" and ops[lp].attrs.get("out_dtype") == "float32":
            # a metric over the uncast label is the same AUC (Session.fuse_towers)
            attrs["label_alias"] = ops[lp].inputs["X"][0].name
        fused = _synthetic(mop.block, "__ctr_tower", ins, {"Pred": sg.outputs["Out"], "Loss": rm.outputs["Out"]},
                           attrs)
        out[m] = fused
        removed.update({d, types["sigmoid"], types["sigmoid_cross_entropy_with_logits"], xu[0]})
        notes.append("data_norm + __fused_mlp + sigmoid/log-loss -> __ctr_tower")
    return [op for k, op in enumerate(out) if k not in removed]


def lower(program: Program, fetch_names=(), gpu: bool = True, engine_cvm_offset: int = 2,
          fuse: bool = True) -> Lowered:
    all_ops = list(program.global_block().ops)
    ops = [op for op in all_ops if not op.attrs.get("op_role")]
    bwd = [op for op in all_ops if op.attrs.get("op_role") == 1]
    opt = [op for op in all_ops if op.attrs.get("op_role") == 2]
    fetch = set(fetch_names)
    notes: List[str] = []
    storage: Dict[str, StorageSpec] = {}
    if fuse:
        ops = _fuse_pull_seqpool(ops, fetch, engine_cvm_offset, notes)
        ops = _absorb_concat(ops, notes)
        if gpu:
            from .kernels import _fc_fp32

            ops = _fuse_cvm(ops, fetch, notes)
            ops = _fuse_mlp(ops, fetch, storage, notes)
            ops = _fuse_tower(ops, fetch, notes, fp32=_fc_fp32())
    for op in ops + bwd + opt:
        if op.type not in KERNELS:
            raise NotImplementedError(f"no kernel for op '{op.type}'")
    return Lowered(ops, storage, notes, bwd, opt)
