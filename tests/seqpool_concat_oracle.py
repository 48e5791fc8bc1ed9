"""numpy transcription of the reference fused_seqpool_cvm pooling + CVM
(paddle/fluid/operators/fused/fused_seqpool_cvm_op.cu: the quant / filter /
embed-filter / embedx_concate kernels at 35-365 and FusedCVMKernelWithCVM* at
371-425), written loop-for-loop from the kernel text, used as the oracle of
the embedx_concate_filter matrix (no reference fixture covers it: parity
unpinned beyond the kernel text)."""
import math

import numpy as np


def ref_fused_seqpool_cvm(xs, offs, B, *, pad_value=0.0, need_filter=False, embed_threshold_filter=False,
                          show_coeff=0.2, clk_coeff=1.0, threshold=0.96, embed_threshold=0.0, cvm_offset=2,
                          quant_ratio=0, embed_thres_size=0, embedx_concate_size=1,
                          embedx_concate_filter=False):
    """use_cvm=True, clk_filter=False. xs[s]: [L_s, E] float64, offs[s]: [B+1]."""
    if quant_ratio == 0 and need_filter:
        quant_ratio = 128  # python layer default (contrib/layers/nn.py)
    ecs = embedx_concate_size
    outs = []
    for x, off in zip(xs, offs):
        L, E = x.shape
        ets = embed_thres_size if embed_thres_size else E - cvm_offset

        def flag(k):  # KernelEmbedQuantFilter
            show, click = x[k, 0], x[k, 1]
            if (show - click) * show_coeff + click * clk_coeff < threshold:
                return 0
            emb = x[k, cvm_offset:]
            score = math.sqrt(sum(emb[i] * emb[i] for i in range(1, ets))) + abs(emb[0])
            return 0 if score < embed_threshold else 1

        def sc_keep(k):
            show, click = x[k, 0], x[k, 1]
            return not ((show - click) * show_coeff + click * clk_coeff < threshold)

        def qv(k, e):
            v = x[k, e]
            if e < cvm_offset:
                return v
            return int(v * quant_ratio + 0.5) / float(quant_ratio)

        pooled = np.zeros((B, ecs, E))
        for b in range(B):
            start, end = int(off[b]), int(off[b + 1])
            for j in range(ecs):
                if ecs == 1:
                    rng = range(start, end)
                else:
                    rng = range(start + j, min(start + j + 1, end))
                for e in range(E):
                    val = pad_value
                    for k in rng:
                        if quant_ratio > 0:
                            if need_filter:
                                if embed_threshold_filter:
                                    if (ecs == 1 or embedx_concate_filter) and flag(k) == 0:
                                        continue
                                elif (ecs == 1 or embedx_concate_filter) and not sc_keep(k):
                                    continue
                            val += qv(k, e)
                        else:  # FusedSeqpoolKernelNormal
                            val += x[k, e]
                    pooled[b, j, e] = val
        out = pooled.copy()
        out[:, :, 0] = np.log(pooled[:, :, 0] + 1)
        out[:, :, 1] = np.log(pooled[:, :, 1] + 1) - np.log(pooled[:, :, 0] + 1)
        outs.append(out.reshape(B, ecs * E))
    return outs
