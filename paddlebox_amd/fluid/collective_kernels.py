"""Stock collective ops of a fluid program (reference ``ops/collective/``:
``c_allreduce_{sum,max,min,prod}``, ``c_allreduce_xsum``, ``c_reduce_sum``,
``c_broadcast``, ``c_allgather``, ``c_mixallgather``, ``c_sync_*_stream``,
``c_comm_init*`` / ``c_gen_nccl_id``) on the session's process group (RCCL
on the GPU, gloo on the CPU).  One process per GPU, so the reference's
per-device rings are ranks here; ``nranks`` of c_mixallgather is the node
count and the node size comes from the launcher (LOCAL_WORLD_SIZE)."""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel.comm import allreduce_sum
from .kernels import _val, kernel


def _group(ctx):
    return ctx.group


def _active(ctx) -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(_group(ctx)) > 1


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
        "prod": dist.ReduceOp.PRODUCT}


def _allreduce(ctx, op, red):
    x = _val(ctx.get(op.inputs["X"][0]))
    out = x.detach().clone()
    if _active(ctx):
        if red == "sum":
            # the session's self-tested IPC mesh (one collective kernel,
            # graph-capturable) when it has one, else RCCL / gloo
            allreduce_sum(out, _group(ctx))
        else:
            dist.all_reduce(out, op=_OPS[red], group=_group(ctx))
    ctx.set(op.outputs["Out"][0], out)


for _r in _OPS:
    kernel(f"c_allreduce_{_r}")(lambda ctx, op, _r=_r: _allreduce(ctx, op, _r))


@kernel("coalesce_tensor")
def k_coalesce_tensor(ctx, op):
    """Fused view of many tensors (coalesce_tensor_op.cc).  When the inputs
    are consecutive fp32 slices of one buffer -- gradients in the dense arena
    -- the fused output is a view of that span (no copy); otherwise a packed
    copy.  The executor writes a rewritten fused value back into the inputs
    (``ctx.cache["coalesced"]``)."""
    xs = [_val(ctx.get(v)) for v in op.inputs["Input"]]
    fused = _span(xs)
    if fused is None:
        fused = torch.cat([x.detach().reshape(-1).float() for x in xs]) if xs else torch.zeros(0)
    out = op.outputs["FusedOutput"][0]
    ctx.set(out, fused)
    ctx.cache.setdefault("coalesced", {})[out.name] = [v.name for v in op.inputs["Input"]]


def _span(xs):
    if not xs or any(x.dtype != torch.float32 or not x.is_contiguous() for x in xs):
        return None
    base = xs[0]
    ptr = base.data_ptr()
    for x in xs:
        if x.untyped_storage().data_ptr() != base.untyped_storage().data_ptr() or x.data_ptr() != ptr:
            return None
        ptr += x.numel() * 4
    total = sum(x.numel() for x in xs)
    return torch.as_strided(base.detach(), (total,), (1,))


@kernel("c_allreduce_xsum")
def k_c_allreduce_xsum(ctx, op):
    """Grouped multi-tensor all-reduce: one fused buffer (c_allreduce_x_op.cc)."""
    xs = [_val(ctx.get(v)).detach() for v in op.inputs["X"]]
    flat = torch.cat([x.reshape(-1).float() for x in xs]) if xs else torch.zeros(0)
    if _active(ctx) and flat.numel():
        allreduce_sum(flat, _group(ctx))
    off = 0
    for v, x in zip(op.outputs["Out"], xs):
        ctx.set(v, flat[off:off + x.numel()].view_as(x).to(x.dtype))
        off += x.numel()


@kernel("c_reduce_sum")
def k_c_reduce_sum(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).detach().clone()
    if _active(ctx):
        dist.reduce(x, dst=int(op.attrs.get("root_id", 0)), group=_group(ctx))
    ctx.set(op.outputs["Out"][0], x)


@kernel("c_broadcast")
def k_c_broadcast(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).detach().clone()
    if _active(ctx):
        dist.broadcast(x, src=int(op.attrs.get("root", 0)), group=_group(ctx))
    ctx.set(op.outputs["Out"][0], x)


@kernel("c_allgather")
def k_c_allgather(ctx, op):
    """[world * d0, ...] in rank order (c_allgather_op)."""
    x = _val(ctx.get(op.inputs["X"][0])).detach().contiguous()
    if _active(ctx):
        w = dist.get_world_size(_group(ctx))
        parts = [torch.empty_like(x) for _ in range(w)]
        dist.all_gather(parts, x, group=_group(ctx))
        x = torch.cat(parts, 0)
    ctx.set(op.outputs["Out"][0], x)


@kernel("c_mixallgather")
def k_c_mixallgather(ctx, op):
    """Fused dense sync (c_mixallgather_op.cc:122-327): the inputs are packed
    into one buffer, then
      nccl_mode 0  all-reduce (hierarchical when nranks > 1: node
                   reduce-scatter -> cross-node shard all-reduce -> node
                   all-gather);
      nccl_mode 1  mix all-gather: node-summed buffers of every node,
                   [nranks * numel] in node order;
      nccl_mode 2  all-gather: every rank's buffer, [world * numel] in rank order."""
    from ..parallel.dense import HierarchicalAllReduce

    xs = [_val(ctx.get(v)).detach().reshape(-1) for v in op.inputs["Input"]]
    buf = torch.cat([x.float() for x in xs]) if xs else torch.zeros(0)
    mode = int(op.attrs.get("nccl_mode", 0))
    nodes = max(1, int(op.attrs.get("nranks", 1)))
    if _active(ctx):
        g = _group(ctx)
        w = dist.get_world_size(g)
        if mode == 0:
            if nodes > 1:
                cache = ctx.cache.setdefault("hier_allreduce", {})
                key = (id(g), w // nodes)
                if key not in cache:
                    cache[key] = HierarchicalAllReduce(g, w // nodes)
                cache[key].allreduce_(buf)
            else:
                dist.all_reduce(buf, group=g)
        elif mode == 2:
            parts = [torch.empty_like(buf) for _ in range(w)]
            dist.all_gather(parts, buf, group=g)
            buf = torch.cat(parts)
        else:
            per_node = max(1, w // nodes)
            parts = [torch.empty_like(buf) for _ in range(w)]
            dist.all_gather(parts, buf, group=g)
            buf = torch.cat([torch.stack(parts[n * per_node:(n + 1) * per_node]).sum(0) for n in range(nodes)])
    elif mode == 1 and nodes > 1:
        raise RuntimeError("c_mixallgather: nranks > 1 needs an initialised process group")
    ctx.set(op.outputs["Output"][0], buf)


@kernel("c_sync_calc_stream", "c_sync_comm_stream")
def k_c_sync_stream(ctx, op):
    """Collectives here are stream-ordered with the compute stream (RCCL on
    the current stream), so the stream syncs only forward their inputs."""
    for src, dst in zip(op.inputs.get("X", []), op.outputs.get("Out", [])):
        ctx.set(dst, ctx.get(src))


@kernel("c_comm_init_all", "c_comm_init", "c_comm_init_multitrainer", "c_gen_nccl_id")
def k_c_comm_init(ctx, op):
    """Communicator setup is the launcher's (torchrun + init_process_group);
    the ops are accepted as no-ops."""
    return None
