"""``fluid.layers`` used by PaddleBox CTR programs.

Each function only records an op into the default main program (and the
parameter initialisers into the startup program); kernels live in
``paddlebox_amd/fluid/kernels.py``.  Signatures follow the reference
(``py/fluid/layers/nn.py``: ``fc`` :243, ``_pull_cache_value`` :779,
``_pull_box_sparse`` :793-840, ``lookup_input`` :843, ``_store_q_value`` :857,
``data_norm`` :3490-3676, ``masked_data_norm`` :3677,
``continuous_value_model`` :14947).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np

from .. import initializer as I
from ..framework import ParamAttr, Variable, default_main_program
from ..layer_helper import LayerHelper


def _as_list(x) -> List[Variable]:
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _batch_shape(*dims) -> tuple:
    return (-1,) + tuple(int(d) for d in dims)


# ----------------------------------------------------------------- inputs
def data(name: str, shape: Sequence[int], dtype="float32", lod_level: int = 0, append_batch_size: bool = True,
         type=None, stop_gradient: bool = True) -> Variable:  # noqa: A002
    shape = list(shape)
    if append_batch_size:
        shape = [-1] + shape
    blk = default_main_program().global_block()
    return blk.create_var(name, shape, dtype, lod_level, stop_gradient=stop_gradient, is_data=True)


# ----------------------------------------------------------------- dense layers
def fc(input, size: int, num_flatten_dims: int = 1, param_attr=None, bias_attr=None, act=None,  # noqa: A002
       name=None) -> Variable:
    """Fully connected; weight ``[in, size]`` (fluid layout).  Multiple inputs
    are summed (each with its own weight), as in the reference."""
    helper = LayerHelper("fc", name)
    ins = _as_list(input)
    pattrs = param_attr if isinstance(param_attr, (list, tuple)) else [param_attr] * len(ins)
    muls = []
    for x, pa in zip(ins, pattrs):
        in_dim = int(np.prod([d for d in x.shape[num_flatten_dims:]]))
        w = helper.create_parameter(pa, [in_dim, size], x.dtype)
        out = helper.create_variable_for_type_inference(x.dtype, _batch_shape(size))
        muls.append((x, w, out))
    b = helper.create_parameter(bias_attr, [size], ins[0].dtype, is_bias=True)
    if len(muls) == 1:
        x, w, out = muls[0]
        helper.append_op("fc", {"Input": [x], "W": [w], "Bias": [b] if b is not None else []},
                         {"Out": [out]}, {"in_num_col_dims": num_flatten_dims,
                                          "activation_type": act or ""})
        return out
    parts = []
    for x, w, out in muls:
        helper.append_op("fc", {"Input": [x], "W": [w], "Bias": []}, {"Out": [out]},
                         {"in_num_col_dims": num_flatten_dims, "activation_type": ""})
        parts.append(out)
    s = sums(parts)
    if b is not None:
        s = _elementwise("elementwise_add", s, b, axis=1)
    return helper.append_activation(s, act)


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,  # noqa: A002
              dtype="float32"):
    helper = LayerHelper("embedding")
    w = helper.create_parameter(param_attr, list(size), dtype)
    out = helper.create_variable_for_type_inference(dtype, _batch_shape(size[1]), input.lod_level)
    helper.append_op("lookup_table", {"Ids": [input], "W": [w]}, {"Out": [out]},
                     {"padding_idx": -1 if padding_idx is None else int(padding_idx)})
    return out


def _unary(op_type, x, attrs=None, name=None):
    helper = LayerHelper(op_type, name)
    out = helper.create_variable_for_type_inference(x.dtype, x.shape, x.lod_level)
    helper.append_op(op_type, {"X": [x]}, {"Out": [out]}, attrs or {})
    return out


def relu(x, name=None):
    return _unary("relu", x, name=name)


def sigmoid(x, name=None):
    return _unary("sigmoid", x, name=name)


def tanh(x, name=None):
    return _unary("tanh", x, name=name)


def exp(x, name=None):
    return _unary("exp", x, name=name)


def log(x, name=None):
    return _unary("log", x, name=name)


def sqrt(x, name=None):
    return _unary("sqrt", x, name=name)


def square(x, name=None):
    return _unary("square", x, name=name)


def abs(x, name=None):  # noqa: A001
    return _unary("abs", x, name=name)


def softmax(input, axis=-1, name=None, use_cudnn=False):  # noqa: A002
    return _unary("softmax", input, {"axis": axis}, name)


def leaky_relu(x, alpha=0.02, name=None):
    return _unary("leaky_relu", x, {"alpha": alpha}, name)


def clip(x, min, max, name=None):  # noqa: A002
    return _unary("clip", x, {"min": float(min), "max": float(max)}, name)


def dropout(x, dropout_prob, is_test=False, seed=None, name=None,
            dropout_implementation="downgrade_in_infer"):
    return _unary("dropout", x, {"dropout_prob": float(dropout_prob), "is_test": is_test,
                                 "dropout_implementation": dropout_implementation}, name)


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    out = _unary("scale", x, {"scale": float(scale), "bias": float(bias), "bias_after_scale": bias_after_scale},
                 name)
    return LayerHelper("scale").append_activation(out, act)


def cast(x, dtype):
    helper = LayerHelper("cast")
    out = helper.create_variable_for_type_inference(dtype, x.shape, x.lod_level)
    helper.append_op("cast", {"X": [x]}, {"Out": [out]}, {"out_dtype": out.dtype})
    return out


def _elementwise(op_type, x, y, axis=-1, act=None, name=None):
    helper = LayerHelper(op_type, name)
    out = helper.create_variable_for_type_inference(x.dtype, x.shape, x.lod_level)
    helper.append_op(op_type, {"X": [x], "Y": [y]}, {"Out": [out]}, {"axis": axis})
    return helper.append_activation(out, act)


def elementwise_add(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_add", x, y, axis, act, name)


def elementwise_sub(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_sub", x, y, axis, act, name)


def elementwise_mul(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_mul", x, y, axis, act, name)


def elementwise_div(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_div", x, y, axis, act, name)


def elementwise_max(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_max", x, y, axis, act, name)


def elementwise_min(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_min", x, y, axis, act, name)


def elementwise_pow(x, y, axis=-1, act=None, name=None):
    return _elementwise("elementwise_pow", x, y, axis, act, name)


def sums(input, out=None):  # noqa: A002
    helper = LayerHelper("sum")
    ins = _as_list(input)
    out = out or helper.create_variable_for_type_inference(ins[0].dtype, ins[0].shape)
    helper.append_op("sum", {"X": ins}, {"Out": [out]})
    return out


def matmul(x, y, transpose_x=False, transpose_y=False, alpha=1.0, name=None):
    helper = LayerHelper("matmul", name)
    out = helper.create_variable_for_type_inference(x.dtype)
    helper.append_op("matmul", {"X": [x], "Y": [y]}, {"Out": [out]},
                     {"transpose_X": transpose_x, "transpose_Y": transpose_y, "alpha": float(alpha)})
    return out


def mul(x, y, x_num_col_dims=1, y_num_col_dims=1, name=None):
    helper = LayerHelper("mul", name)
    out = helper.create_variable_for_type_inference(x.dtype)
    helper.append_op("mul", {"X": [x], "Y": [y]}, {"Out": [out]},
                     {"x_num_col_dims": x_num_col_dims, "y_num_col_dims": y_num_col_dims})
    return out


def concat(input, axis=0, name=None):  # noqa: A002
    helper = LayerHelper("concat", name)
    ins = _as_list(input)
    width = None
    if axis in (1, -1) and all(len(v.shape) == 2 and v.shape[1] > 0 for v in ins):
        width = sum(v.shape[1] for v in ins)
    out = helper.create_variable_for_type_inference(ins[0].dtype, _batch_shape(width) if width else ())
    helper.append_op("concat", {"X": ins}, {"Out": [out]}, {"axis": axis})
    return out


def split(input, num_or_sections, dim=-1, name=None):  # noqa: A002
    helper = LayerHelper("split", name)
    n = num_or_sections if isinstance(num_or_sections, int) else len(num_or_sections)
    outs = [helper.create_variable_for_type_inference(input.dtype) for _ in range(n)]
    helper.append_op("split", {"X": [input]}, {"Out": outs},
                     {"num": num_or_sections if isinstance(num_or_sections, int) else 0,
                      "sections": [] if isinstance(num_or_sections, int) else list(num_or_sections),
                      "axis": dim})
    return outs


def slice(input, axes, starts, ends):  # noqa: A001,A002
    helper = LayerHelper("slice")
    out = helper.create_variable_for_type_inference(input.dtype)
    helper.append_op("slice", {"Input": [input]}, {"Out": [out]},
                     {"axes": list(axes), "starts": list(starts), "ends": list(ends)})
    return out


def reshape(x, shape, actual_shape=None, act=None, inplace=False, name=None):
    helper = LayerHelper("reshape2", name)
    out = helper.create_variable_for_type_inference(x.dtype, tuple(shape))
    helper.append_op("reshape2", {"X": [x]}, {"Out": [out]}, {"shape": list(shape)})
    return helper.append_activation(out, act)


def transpose(x, perm, name=None):
    return _unary("transpose2", x, {"axis": list(perm)}, name)


def squeeze(input, axes, name=None):  # noqa: A002
    return _unary("squeeze2", input, {"axes": list(axes)}, name)


def unsqueeze(input, axes, name=None):  # noqa: A002
    return _unary("unsqueeze2", input, {"axes": list(axes)}, name)


def stack(x, axis=0, name=None):
    helper = LayerHelper("stack", name)
    out = helper.create_variable_for_type_inference(x[0].dtype)
    helper.append_op("stack", {"X": list(x)}, {"Y": [out]}, {"axis": axis})
    return out


def fill_constant(shape, dtype, value, force_cpu=False, out=None, name=None):
    helper = LayerHelper("fill_constant", name)
    out = out or helper.create_variable_for_type_inference(dtype, tuple(shape))
    out.stop_gradient = True
    helper.append_op("fill_constant", {}, {"Out": [out]},
                     {"shape": list(shape), "dtype": out.dtype, "value": float(value)})
    return out


def fill_constant_batch_size_like(input, shape, dtype, value, input_dim_idx=0, output_dim_idx=0,  # noqa: A002
                                  force_cpu=False):
    helper = LayerHelper("fill_constant_batch_size_like")
    out = helper.create_variable_for_type_inference(dtype, tuple(shape))
    out.stop_gradient = True
    helper.append_op("fill_constant_batch_size_like", {"Input": [input]}, {"Out": [out]},
                     {"shape": list(shape), "dtype": out.dtype, "value": float(value),
                      "input_dim_idx": input_dim_idx, "output_dim_idx": output_dim_idx})
    return out


def zeros_like(x, out=None):
    return _unary("fill_zeros_like", x)


def ones_like(x, out=None):
    return _unary("fill_ones_like", x)


def assign(input, output=None):  # noqa: A002
    return _unary("assign", input)


def reduce_sum(input, dim=None, keep_dim=False, name=None):  # noqa: A002
    return _unary("reduce_sum", input, {"dim": dim, "keep_dim": keep_dim}, name)


def reduce_mean(input, dim=None, keep_dim=False, name=None):  # noqa: A002
    return _unary("reduce_mean", input, {"dim": dim, "keep_dim": keep_dim}, name)


def reduce_max(input, dim=None, keep_dim=False, name=None):  # noqa: A002
    return _unary("reduce_max", input, {"dim": dim, "keep_dim": keep_dim}, name)


def mean(x, name=None):
    return _unary("mean", x, name=name)


def log_loss(input, label, epsilon=1e-4, name=None):  # noqa: A002
    helper = LayerHelper("log_loss", name)
    out = helper.create_variable_for_type_inference(input.dtype, input.shape)
    helper.append_op("log_loss", {"Predicted": [input], "Labels": [label]}, {"Loss": [out]},
                     {"epsilon": float(epsilon)})
    return out


def sigmoid_cross_entropy_with_logits(x, label, ignore_index=-100, name=None, normalize=False):
    helper = LayerHelper("sigmoid_cross_entropy_with_logits", name)
    out = helper.create_variable_for_type_inference(x.dtype, x.shape)
    helper.append_op("sigmoid_cross_entropy_with_logits", {"X": [x], "Label": [label]}, {"Out": [out]},
                     {"ignore_index": ignore_index, "normalize": normalize})
    return out


def cross_entropy(input, label, soft_label=False, ignore_index=-100):  # noqa: A002
    helper = LayerHelper("cross_entropy")
    out = helper.create_variable_for_type_inference(input.dtype, _batch_shape(1))
    helper.append_op("cross_entropy", {"X": [input], "Label": [label]}, {"Y": [out]},
                     {"soft_label": soft_label, "ignore_index": ignore_index})
    return out


def square_error_cost(input, label):  # noqa: A002
    return square(_elementwise("elementwise_sub", input, label))


def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):  # noqa: A002
    return _unary("sequence_pool", input, {"pooltype": pool_type.upper(), "pad_value": float(pad_value)})


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1):  # noqa: A002
    """In-graph streaming AUC (phi auc kernel); returns
    (auc, batch_auc, [stat_pos, stat_neg, ...]) like the reference."""
    helper = LayerHelper("auc")
    auc_out = helper.create_variable_for_type_inference("float64", (1,))
    batch_auc_out = helper.create_variable_for_type_inference("float64", (1,))
    stat_pos = helper.create_global_variable(shape=[num_thresholds + 1], dtype="float64")
    stat_neg = helper.create_global_variable(shape=[num_thresholds + 1], dtype="float64")
    helper.append_op("auc", {"Predict": [input], "Label": [label], "StatPos": [stat_pos], "StatNeg": [stat_neg]},
                     {"AUC": [auc_out], "BatchAUC": [batch_auc_out]},
                     {"num_thresholds": num_thresholds, "curve": curve})
    return auc_out, batch_auc_out, [stat_pos, stat_neg, stat_pos, stat_neg]


# ----------------------------------------------------------------- PaddleBox sparse
def _pull_box_sparse(input, size, dtype="float32", offset=0, slot_idx=-1):  # noqa: A002
    """Pull per-occurrence records ``[L_s, size]`` for each slot from BoxPS.
    The gradient of this op IS the sparse update (``push_box_sparse``)."""
    if dtype != "float32":
        raise ValueError("BoxPS only supports float32 embeddings, got " + str(dtype))
    helper = LayerHelper("pull_box_sparse")
    ins = _as_list(input)
    outs = [helper.create_variable_for_type_inference(dtype, (-1, size), v.lod_level) for v in ins]
    helper.append_op("pull_box_sparse", {"Ids": ins}, {"Out": outs},
                     {"size": int(size), "offset": int(offset), "slot_idx": int(slot_idx)})
    return outs[0] if len(outs) == 1 else outs


pull_box_sparse = _pull_box_sparse


def _pull_cache_value(input, size, dtype="float32"):  # noqa: A002
    helper = LayerHelper("pull_cache_value")
    out = helper.create_variable_for_type_inference(dtype, (-1, size))
    helper.append_op("pull_cache_value", {"Id": [input]}, {"Out": [out]}, {"size": int(size)})
    return out


def lookup_input(input, size):  # noqa: A002
    helper = LayerHelper("lookup_input")
    out = helper.create_variable_for_type_inference("float32", (-1, size))
    helper.append_op("lookup_input", {"Id": [input]}, {"Out": [out]}, {"size": int(size)})
    return out


def _store_q_value(input, dtype="float32"):  # noqa: A002
    helper = LayerHelper("store_q_value")
    helper.append_op("store_q_value", {"Ids": _as_list(input)}, {}, {})


def continuous_value_model(input, cvm, use_cvm=True):  # noqa: A002
    helper = LayerHelper("cvm")
    w = input.shape[-1] if input.shape else -1
    out = helper.create_variable_for_type_inference(input.dtype, (-1, w if use_cvm or w < 0 else w - 2),
                                                    input.lod_level)
    helper.append_op("cvm", {"X": [input], "CVM": [cvm]}, {"Y": [out]}, {"use_cvm": use_cvm})
    return out


def _data_norm_params(helper, input, param_attr, enable_scale_and_shift, extra_dims=None):
    C = input.shape[-1] if extra_dims is None else extra_dims
    pa = param_attr or {}
    bs_default = pa.get("batch_size", 1e4)
    bsum_default = pa.get("batch_sum", 0.0)
    bsq_default = pa.get("batch_square", 1e4)
    name = helper.name

    def mk(suffix, v):
        return helper.create_parameter(ParamAttr(name=f"{name}.{suffix}", initializer=I.Constant(v)), [C],
                                       input.dtype)

    bsize = mk("batch_size", bs_default)
    bsum = mk("batch_sum", bsum_default)
    bsq = mk("batch_square_sum", bsq_default)
    for p in (bsize, bsum, bsq):
        p.is_summary = True  # updated by the op's backward, not by the optimizer
    scale_w = bias = None
    if enable_scale_and_shift:
        scale_w = mk("scale_w", pa.get("scale_w", 1.0))
        bias = mk("bias", pa.get("bias", 0.0))
    return bsize, bsum, bsq, scale_w, bias


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout="NCHW", in_place=False,  # noqa: A002
              name=None, moving_mean_name=None, moving_variance_name=None, do_model_average_for_mean_and_var=True,
              slot_dim=-1, sync_stats=False, update_norm=True, summary_decay_rate=0.9999999,
              enable_scale_and_shift=False):
    helper = LayerHelper("data_norm", name)
    bsize, bsum, bsq, scale_w, bias = _data_norm_params(helper, input, param_attr, enable_scale_and_shift)
    out = helper.create_variable_for_type_inference(input.dtype, input.shape)
    means = helper.create_variable_for_type_inference(input.dtype, stop_gradient=True)
    scales = helper.create_variable_for_type_inference(input.dtype, stop_gradient=True)
    ins = {"X": [input], "BatchSize": [bsize], "BatchSum": [bsum], "BatchSquareSum": [bsq]}
    if enable_scale_and_shift:
        ins["scale_w"] = [scale_w]
        ins["bias"] = [bias]
    helper.append_op("data_norm", ins, {"Y": [out], "Means": [means], "Scales": [scales]},
                     {"epsilon": float(epsilon), "slot_dim": int(slot_dim), "sync_stats": sync_stats,
                      "summary_decay_rate": float(summary_decay_rate), "update_norm": update_norm,
                      "enable_scale_and_shift": enable_scale_and_shift, "is_test": False})
    return helper.append_activation(out, act)


def masked_data_norm(input, mask, act=None, epsilon=1e-05, param_attr=None, data_layout="NCHW",  # noqa: A002
                     in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
                     do_model_average_for_mean_and_var=True, slot_dim=-1, sync_stats=False, update_norm=True,
                     summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    helper = LayerHelper("masked_data_norm", name)
    bsize, bsum, bsq, scale_w, bias = _data_norm_params(helper, input, param_attr, enable_scale_and_shift)
    out = helper.create_variable_for_type_inference(input.dtype, input.shape)
    ins = {"X": [input], "Mask": [mask], "BatchSize": [bsize], "BatchSum": [bsum], "BatchSquareSum": [bsq]}
    if enable_scale_and_shift:
        ins["scale_w"] = [scale_w]
        ins["bias"] = [bias]
    helper.append_op("masked_data_norm", ins, {"Y": [out]},
                     {"epsilon": float(epsilon), "slot_dim": int(slot_dim), "sync_stats": sync_stats,
                      "summary_decay_rate": float(summary_decay_rate), "update_norm": update_norm,
                      "enable_scale_and_shift": enable_scale_and_shift, "is_test": False})
    return helper.append_activation(out, act)


def shuffle_batch(x, seed=None):
    helper = LayerHelper("shuffle_batch")
    out = helper.create_variable_for_type_inference(x.dtype, x.shape)
    helper.append_op("shuffle_batch", {"X": [x]}, {"Out": [out]}, {"startup_seed": int(seed or 0)})
    return out


def partial_concat(input, start_index=0, length=-1):  # noqa: A002
    helper = LayerHelper("partial_concat")
    ins = _as_list(input)
    out = helper.create_variable_for_type_inference(ins[0].dtype)
    helper.append_op("partial_concat", {"X": ins}, {"Out": [out]},
                     {"start_index": int(start_index), "length": int(length)})
    return out


def partial_sum(input, start_index=0, length=-1):  # noqa: A002
    helper = LayerHelper("partial_sum")
    ins = _as_list(input)
    out = helper.create_variable_for_type_inference(ins[0].dtype)
    helper.append_op("partial_sum", {"X": ins}, {"Out": [out]},
                     {"start_index": int(start_index), "length": int(length)})
    return out
