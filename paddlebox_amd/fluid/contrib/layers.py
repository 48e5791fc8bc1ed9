"""``fluid.contrib.layers`` -- the PaddleBox CTR op family.

Signatures follow ``py/fluid/contrib/layers/nn.py`` (rank_attention :1497,
rank_attention2 :1574, batch_fc :1605, _pull_box_extended_sparse :1678,
fused_seqpool_cvm :1750, ..._with_diff_thres :1833, ..._with_conv :1912,
..._with_pcoc :1979, ..._tradew :2049, ..._with_credit :2107,
cross_norm_layer_hadamard :2163, scaled_fc :2587, scaled_int8fc :2648,
fused_seqpool_concat :2726, fused_concat :2795, fused_seq_tensor :2834).
Kernels: ``paddlebox_amd/fluid/kernels.py`` -> ``paddlebox_amd/ops``.
"""
from __future__ import annotations

import numpy as np

from .. import initializer as I
from ..framework import ParamAttr
from ..layer_helper import LayerHelper
from ..layers.nn import _as_list, partial_concat, partial_sum, shuffle_batch  # noqa: F401


def _seqpool_out_width(E, use_cvm, cvm_offset, clk_filter=False, embed_thres_size=0, concat=1):
    if E is None or E < 0:
        return -1
    if use_cvm:
        return (E - 1 if clk_filter else E) * concat
    return (E - cvm_offset - embed_thres_size) * concat


def _seqpool_family(op_type, input, cvm, attrs, out_width_fn, extra_inputs=None):  # noqa: A002
    helper = LayerHelper(op_type)
    ins = _as_list(input)
    outs = []
    for v in ins:
        E = v.shape[-1] if v.shape else -1
        outs.append(helper.create_variable_for_type_inference(v.dtype, (-1, out_width_fn(E))))
    inputs = {"X": ins, "CVM": [cvm]}
    inputs.update(extra_inputs or {})
    helper.append_op(op_type, inputs, {"Out": outs}, attrs)
    return outs


def fused_seqpool_cvm(input, pool_type, cvm, pad_value=0.0, use_cvm=True, need_filter=False,  # noqa: A002
                      embed_threshold_filter=False, show_coeff=0.2, clk_coeff=1.0, threshold=0.96,
                      embed_threshold=0, cvm_offset=2, quant_ratio=0, clk_filter=False, embed_thres_size=0,
                      embedx_concate_size=1, embedx_concate_filter=False, fill_zero=True):
    if pool_type.upper() != "SUM":
        raise ValueError("fused_seqpool_cvm only supports SUM pooling, got " + pool_type)
    if quant_ratio == 0 and need_filter:
        quant_ratio = 128  # reference default when filtering
    attrs = dict(pooltype="SUM", pad_value=float(pad_value), use_cvm=use_cvm, cvm_offset=int(cvm_offset),
                 need_filter=need_filter, embed_threshold_filter=embed_threshold_filter,
                 show_coeff=float(show_coeff), clk_coeff=float(clk_coeff), threshold=float(threshold),
                 embed_threshold=float(embed_threshold), quant_ratio=int(quant_ratio), clk_filter=clk_filter,
                 embed_thres_size=int(embed_thres_size), embedx_concate_size=int(embedx_concate_size),
                 embedx_concate_filter=embedx_concate_filter, fill_zero=fill_zero)
    return _seqpool_family("fused_seqpool_cvm", input, cvm, attrs,
                           lambda E: _seqpool_out_width(E, use_cvm, cvm_offset, clk_filter, embed_thres_size,
                                                        embedx_concate_size))


def fused_seqpool_cvm_with_diff_thres(input, pool_type, cvm, pad_value=0.0, use_cvm=True,  # noqa: A002
                                      need_filter=False, show_coeff=0.2, clk_coeff=1.0, threshold=0.96,
                                      cvm_offset=2, quant_ratio=0, clk_filter=False, xbox_diff_thres_filter=False,
                                      threshold_vec=()):
    if quant_ratio == 0 and need_filter:
        quant_ratio = 128
    attrs = dict(pooltype="SUM", pad_value=float(pad_value), use_cvm=use_cvm, cvm_offset=int(cvm_offset),
                 need_filter=need_filter, show_coeff=float(show_coeff), clk_coeff=float(clk_coeff),
                 threshold=float(threshold), quant_ratio=int(quant_ratio), clk_filter=clk_filter,
                 xbox_diff_thres_filter=xbox_diff_thres_filter, threshold_vec=[float(t) for t in threshold_vec])
    return _seqpool_family("fused_seqpool_cvm_with_diff_thres", input, cvm, attrs,
                           lambda E: _seqpool_out_width(E, use_cvm, cvm_offset, clk_filter))


def fused_seqpool_cvm_with_conv(input, pool_type, cvm, pad_value=0.0, use_cvm=True, need_filter=False,  # noqa: A002
                                show_coeff=0.2, clk_coeff=1.0, threshold=0.96, show_filter=False, cvm_offset=3,
                                embedx_concate_size=1):
    attrs = dict(pooltype="SUM", pad_value=float(pad_value), use_cvm=use_cvm, cvm_offset=int(cvm_offset),
                 need_filter=need_filter, show_coeff=float(show_coeff), clk_coeff=float(clk_coeff),
                 threshold=float(threshold), show_filter=show_filter, embedx_concate_size=int(embedx_concate_size))
    return _seqpool_family("fused_seqpool_cvm_with_conv", input, cvm, attrs,
                           lambda E: -1 if E < 0 else ((E - 1 if show_filter else E) if use_cvm
                                                       else E - cvm_offset) * embedx_concate_size)


def fused_seqpool_cvm_with_pcoc(input, pool_type, pcoc_cvm, pad_value=0.0, use_cvm=True,  # noqa: A002
                                need_filter=False, show_coeff=0.2, clk_coeff=1.0, threshold=0.96, cvm_offset=7,
                                max_cvm_offset=7, quant_ratio=0):
    attrs = dict(pooltype="SUM", pad_value=float(pad_value), use_cvm=use_cvm, cvm_offset=int(cvm_offset),
                 max_cvm_offset=int(max_cvm_offset), need_filter=need_filter, show_coeff=float(show_coeff),
                 clk_coeff=float(clk_coeff), threshold=float(threshold), quant_ratio=int(quant_ratio))
    return _seqpool_family("fused_seqpool_cvm_with_pcoc", input, pcoc_cvm, attrs,
                           lambda E: -1 if E < 0 else (E - (max_cvm_offset - 2 * cvm_offset + 6) if use_cvm
                                                       else E - max_cvm_offset))


def fused_seqpool_cvm_tradew(input, pool_type, cvm, pad_value=0.0, use_cvm=True, cvm_offset=2,  # noqa: A002
                             trade_id=-1, trade_num=2):
    attrs = dict(pooltype="SUM", pad_value=float(pad_value), use_cvm=use_cvm, cvm_offset=int(cvm_offset),
                 trade_id=int(trade_id), trade_num=int(trade_num))
    return _seqpool_family("fused_seqpool_cvm_tradew", input, cvm, attrs,
                           lambda E: -1 if E < 0 else ((E - trade_num) if use_cvm else E - cvm_offset - trade_num))


def fused_seqpool_cvm_with_credit(input, pool_type, cvm, pad_value=0.0, use_cvm=True, show_filter=False,  # noqa: A002
                                  cvm_offset=4):
    attrs = dict(pooltype="SUM", pad_value=float(pad_value), use_cvm=use_cvm, cvm_offset=int(cvm_offset),
                 show_filter=show_filter)
    return _seqpool_family("fused_seqpool_cvm_with_credit", input, cvm, attrs,
                           lambda E: -1 if E < 0 else ((E - 1 if show_filter else E) if use_cvm
                                                       else E - cvm_offset))


def _pull_box_extended_sparse(input, size, extend_size=64, dtype="float32", mask=(), offset=0,  # noqa: A002
                              expand_only=True):
    helper = LayerHelper("pull_box_extended_sparse")
    ins = _as_list(input)
    mask = list(mask)
    if not mask:
        outs = [helper.create_variable_for_type_inference(dtype, (-1, size)) for _ in ins]
        outs_ex = [helper.create_variable_for_type_inference(dtype, (-1, extend_size)) for _ in ins]
    else:
        outs, outs_ex = [], []
        for flag in mask:
            if flag & 1:
                outs.append(helper.create_variable_for_type_inference(dtype, (-1, size)))
            if flag & 2:
                outs_ex.append(helper.create_variable_for_type_inference(dtype, (-1, extend_size)))
    helper.append_op("pull_box_extended_sparse", {"Ids": ins}, {"Out": outs, "OutExtend": outs_ex},
                     {"emb_size": int(size), "emb_extended_size": int(extend_size), "mask": mask,
                      "offset": int(offset), "expand_only": expand_only})
    if len(outs) == 1 and len(outs_ex) == 1:
        return outs[0], outs_ex[0]
    return outs, outs_ex


def cross_norm_layer_hadamard(input, fields_num, embed_dim, param_dict={}, summary_decay_rate=0.9999999,  # noqa: A002,B006
                              epsilon=1e-04, name=None, sync_stats=False):
    helper = LayerHelper("cross_norm_hadamard", name)
    width = fields_num * (3 * embed_dim + 1)
    layer = np.zeros((3, width), dtype=np.float32)
    layer[0, :] = param_dict.get("batch_size", 1e4)
    layer[1, :] = param_dict.get("batch_sum", 0.0)
    layer[2, :] = param_dict.get("batch_square", 1e4)
    summary = helper.create_parameter(ParamAttr(name=f"{helper.name}.cross_summary",
                                                initializer=I.NumpyArrayInitializer(layer)), [3, width],
                                      input.dtype)
    summary.is_summary = True
    out = helper.create_variable_for_type_inference(input.dtype, (-1, width))
    helper.append_op("cross_norm_hadamard", {"Input": [input], "SummaryInput": [summary]}, {"Out": [out]},
                     {"fields_num": int(fields_num), "embed_dim": int(embed_dim), "epsilon": float(epsilon),
                      "summary_decay_rate": float(summary_decay_rate), "sync_stats": sync_stats})
    return out


def rank_attention(input, rank_offset, rank_param_shape, rank_param_attr, max_rank=3, max_size=0,  # noqa: A002
                   enable_input_bp=False):
    helper = LayerHelper("rank_attention")
    assert input.shape[1] * max_rank * max_rank == rank_param_shape[0]
    w = helper.create_parameter(rank_param_attr, list(rank_param_shape), input.dtype)
    out = helper.create_variable_for_type_inference(input.dtype, (-1, rank_param_shape[1]))
    helper.append_op("rank_attention", {"X": [input], "RankOffset": [rank_offset], "RankParam": [w]},
                     {"Out": [out]}, {"MaxRank": int(max_rank), "MaxSize": int(max_size),
                                      "EnableInputBp": enable_input_bp})
    return out


def rank_attention2(input, rank_offset, rank_param_shape, rank_param_attr, max_rank=3, max_size=0):  # noqa: A002
    helper = LayerHelper("rank_attention2")
    assert input.shape[1] * max_rank * max_rank == rank_param_shape[0]
    w = helper.create_parameter(rank_param_attr, list(rank_param_shape), input.dtype)
    out = helper.create_variable_for_type_inference(input.dtype, (-1, rank_param_shape[1]))
    helper.append_op("rank_attention2", {"X": [input], "RankOffset": [rank_offset], "RankParam": [w]},
                     {"Out": [out]}, {"MaxRank": int(max_rank), "EnableInputBp": True})
    return out


def batch_fc(input, param_size, param_attr, bias_size, bias_attr, act=None, batchcount=0,  # noqa: A002
             transpose_weight=False):
    helper = LayerHelper("batch_fc")
    if batchcount == 0:
        assert input.shape[0] == param_size[0] and input.shape[2] == param_size[1]
        assert param_size[2] == bias_size[1] and input.shape[0] == bias_size[0]
    w = helper.create_parameter(param_attr, list(param_size), input.dtype)
    b = helper.create_parameter(bias_attr, list(bias_size), input.dtype)
    if batchcount == 0:
        shape = (param_size[0], -1, param_size[2])
    else:
        shape = (-1, (param_size[0] if not transpose_weight else param_size[1]))
    out = helper.create_variable_for_type_inference(input.dtype, shape)
    helper.append_op("batch_fc", {"Input": [input], "W": [w], "Bias": [b]}, {"Out": [out]},
                     {"batchcount": int(batchcount), "transpose_weight": transpose_weight})
    return helper.append_activation(out, act)


def scaled_fc(input, param_size, param_attr, bias_size, bias_attr, input_scale_factor, bias_scale_factor,  # noqa: A002
              grad_scale_factor=256.0, act=None):
    helper = LayerHelper("scaled_fc")
    w = helper.create_parameter(param_attr, list(param_size), input.dtype)
    b = helper.create_parameter(bias_attr, list(bias_size), input.dtype)
    out = helper.create_variable_for_type_inference(input.dtype, (-1, param_size[1]))
    helper.append_op("scaled_fc", {"Input": [input], "W": [w], "Bias": [b]}, {"Out": [out]},
                     {"input_scale_factor": float(input_scale_factor), "bias_scale_factor": float(bias_scale_factor),
                      "grad_scale_factor": float(grad_scale_factor)})
    return helper.append_activation(out, act)


def scaled_int8fc(input, param_size, param_attr, bias_size, bias_attr, input_scale_factor=1.0,  # noqa: A002
                  bias_scale_factor=1.0, grad_scale_factor=1.0, input_expand_factor=1.0, input_clip_factor=2.0,
                  weight_expand_factor=1.0, weight_clip_factor=2.0, int8_range=240.0, act=None):
    helper = LayerHelper("scaled_int8fc")
    w = helper.create_parameter(param_attr, list(param_size), input.dtype)
    b = helper.create_parameter(bias_attr, list(bias_size), input.dtype)
    out = helper.create_variable_for_type_inference(input.dtype, (-1, param_size[1]))
    helper.append_op("scaled_int8fc", {"Input": [input], "W": [w], "Bias": [b]}, {"Out": [out]},
                     {"input_scale_factor": float(input_scale_factor), "bias_scale_factor": float(bias_scale_factor),
                      "grad_scale_factor": float(grad_scale_factor), "input_expand_factor": float(input_expand_factor),
                      "input_clip_factor": float(input_clip_factor),
                      "weight_expand_factor": float(weight_expand_factor),
                      "weight_clip_factor": float(weight_clip_factor), "int8_range": float(int8_range)})
    return helper.append_activation(out, act)


def fused_seqpool_concat(input, offsets=None, dims=None):  # noqa: A002
    """Column-gather concat: group i contributes columns
    ``[offsets[i], offsets[i]+dims[i])`` of each of its inputs; one output per
    position j concatenating ``input[i][j]``'s selected columns over i."""
    helper = LayerHelper("fused_seqpool_concat")
    groups = [_as_list(g) for g in input]
    n = len(groups[0])
    cols = []
    for i, g in enumerate(groups):
        total = g[0].shape[1]
        start = max(0, offsets[i]) if isinstance(offsets, list) and i < len(offsets) else 0
        d = dims[i] if isinstance(dims, list) and i < len(dims) else 0
        if d <= 0:
            d = total - start
        cols.append((start, d))
    width = sum(d for _, d in cols)
    outs = [helper.create_variable_for_type_inference(groups[0][0].dtype, (-1, width)) for _ in range(n)]
    ins = {f"X{i + 1}": g for i, g in enumerate(groups)}
    helper.append_op("fused_seqpool_concat", ins, {"Out": outs},
                     {"col_ranges": [c for c in cols], "n_groups": len(groups)})
    return outs


def fused_concat(input, start_index=0, length=-1, axis=1):  # noqa: A002
    if axis != 1:
        raise ValueError("fused_concat only concatenates columns")
    ins = _as_list(input)
    dim = ins[0].shape[1]
    for v in ins[1:]:
        if v.shape[1] != dim:
            raise ValueError("fused_concat inputs must share their width")
    start_index = max(0, start_index)
    if length <= 0:
        length = dim - start_index
    helper = LayerHelper("fused_concat")
    out = helper.create_variable_for_type_inference(ins[0].dtype, (-1, length * len(ins)))
    helper.append_op("fused_concat", {"X": ins}, {"Out": [out]}, {"offset": start_index, "length": length})
    return out


def fused_seq_tensor(input, batch_count, max_length, slot_num, ad_slot_num, fea_emb_dim, ad_slot_offset):  # noqa: A002
    helper = LayerHelper("fused_seq_tensor")
    dt = input[0].dtype
    din = helper.create_variable_for_type_inference(dt)
    mask = helper.create_variable_for_type_inference(dt)
    side = helper.create_variable_for_type_inference(dt)
    ad_sess = helper.create_variable_for_type_inference(dt)
    helper.append_op("fused_seq_tensor", {"Input": [input[0]], "ADInput": [input[1]]},
                     {"DINOut": [din], "MaskOut": [mask], "SideInfoOut": [side], "ADSlotSessionOut": [ad_sess]},
                     {"batch_count": int(batch_count), "max_length": int(max_length), "slot_num": int(slot_num),
                      "fea_emb_dim": int(fea_emb_dim), "ad_slot_num": int(ad_slot_num),
                      "ad_slot_offset": int(ad_slot_offset)})
    return din, mask, side, ad_sess
