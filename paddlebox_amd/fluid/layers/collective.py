"""fluid.layers.collective (reference ``py/fluid/layers/collective.py``):
program-level collective ops, run by ``fluid/collective_kernels.py``."""
from __future__ import annotations

from typing import Sequence

from ..layer_helper import LayerHelper


def _coll(op_type, x, attrs, shape=None):
    helper = LayerHelper(op_type)
    out = helper.create_variable_for_type_inference(x.dtype, shape if shape is not None else x.shape)
    helper.append_op(op_type, {"X": [x]}, {"Out": [out]}, attrs)
    return out


def _c_allreduce(x, out=None, reduce_type="sum", ring_id=0, use_calc_stream=False):
    if reduce_type not in ("sum", "max", "min", "prod"):
        raise ValueError(f"reduce_type {reduce_type!r}")
    return _coll(f"c_allreduce_{reduce_type}", x, {"ring_id": ring_id, "use_calc_stream": use_calc_stream})


def _c_broadcast(x, root=0, ring_id=0, use_calc_stream=False):
    return _coll("c_broadcast", x, {"root": root, "ring_id": ring_id, "use_calc_stream": use_calc_stream})


def _c_reduce_sum(x, root_id=0, ring_id=0):
    return _coll("c_reduce_sum", x, {"root_id": root_id, "ring_id": ring_id})


def _c_allgather(x, nranks, ring_id=0, use_calc_stream=False):
    shape = (x.shape[0] * nranks,) + tuple(x.shape[1:]) if x.shape and x.shape[0] > 0 else x.shape
    return _coll("c_allgather", x, {"nranks": nranks, "ring_id": ring_id, "use_calc_stream": use_calc_stream},
                 shape)


def _c_sync_calc_stream(x):
    return _coll("c_sync_calc_stream", x, {})


def _c_sync_comm_stream(x, ring_id=0):
    return _coll("c_sync_comm_stream", x, {"ring_id": ring_id})


def _c_allreduce_xsum(xs: Sequence, ring_id=0):
    helper = LayerHelper("c_allreduce_xsum")
    outs = [helper.create_variable_for_type_inference(x.dtype, x.shape) for x in xs]
    helper.append_op("c_allreduce_xsum", {"X": list(xs)}, {"Out": outs}, {"ring_id": ring_id})
    return outs


def _c_mixallgather(xs: Sequence, nranks=1, rankid=0, nccl_mode=0, ring_id=-1):
    """Fused dense sync of several tensors into one buffer (mode 0 all-reduce,
    1 mix all-gather, 2 all-gather)."""
    helper = LayerHelper("c_mixallgather")
    out = helper.create_variable_for_type_inference("float32", (-1,))
    helper.append_op("c_mixallgather", {"Input": list(xs)}, {"Output": [out]},
                     {"nranks": nranks, "rankid": rankid, "nccl_mode": nccl_mode, "ring_id": ring_id})
    return out
