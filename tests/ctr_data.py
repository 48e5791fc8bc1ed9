"""Input generators shared by the CTR op tests (CPU and GPU)."""
import torch


def page_view_ranks(n_pv: int, R: int, gen: torch.Generator, p_single: float = 0.0) -> torch.Tensor:
    """rank_offset [ins, 2R+1] for n_pv page views of 1..R+1 ads each: an ad
    shown at rank r <= R lists every ad of its page view with rank <= R at
    slot r'-1 as (r', instance index); ranks > R are -1 (the layout the
    reference's rank_attention test builds, test_rank_attention_op.py:109).
    A page view holds a single ad with probability ``p_single`` (skews the
    instances towards rank 1)."""
    rows = []
    for _ in range(n_pv):
        n = int(torch.randint(1, R + 2, (1,), generator=gen))
        if p_single and float(torch.rand(1, generator=gen)) < p_single:
            n = 1
        ranks = (torch.randperm(n, generator=gen) + 1).tolist()
        start = len(rows)
        for r in ranks:
            row = [-1] * (2 * R + 1)
            if r <= R:
                row[0] = r
                for k, rk in enumerate(ranks):
                    if rk <= R:
                        row[2 * (rk - 1) + 1] = rk
                        row[2 * (rk - 1) + 2] = start + k
            rows.append(row)
    return torch.tensor(rows, dtype=torch.int32)


def rank_attention_loop(x, ro, W, R):
    """Direct per-instance evaluation of the rank_attention definition."""
    B, C = x.shape
    P = W.shape[1]
    Wb = W.reshape(R * R, C, P)
    out = torch.zeros(B, P, dtype=x.dtype)
    for i in range(B):
        lower = int(ro[i, 0]) - 1
        for k in range(R):
            faster = int(ro[i, 2 * k + 1]) - 1
            idx = int(ro[i, 2 * k + 2])
            if lower < 0 or faster < 0 or idx < 0:
                continue
            out[i] += x[idx] @ Wb[lower * R + faster]
    return out
