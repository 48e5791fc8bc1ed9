"""Synthetic Criteo-shape data (13 dense + 26 sparse slots).

There is no dataset access on the benchmark hosts, so the benchmark and tests
use a generator with Criteo-1TB-like per-slot cardinalities (the public
MLPerf DLRM day-0..23 counts with the 40M cap), scaled so the feature space
totals ``total_features`` (1e9 for the headline config), power-law (Zipf-like)
id popularity per slot, and labels drawn from a hidden logistic model so AUC is
learnable.  Keys are namespaced per slot: ``key = (slot+1) << 44 | id``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import torch

# MLPerf DLRM Criteo-1TB per-feature cardinalities (max_ind_range = 40M)
CRITEO_1TB_CARDINALITIES = [
    39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951, 2953546, 403346, 10, 2208, 11938, 155, 4,
    976, 14, 39979771, 25641295, 39664984, 585935, 12972, 108, 36,
]
NUM_DENSE = 13
NUM_SPARSE = 26
SLOT_SHIFT = 44


def scaled_cardinalities(total_features: int, base: List[int] = CRITEO_1TB_CARDINALITIES) -> List[int]:
    s = sum(base)
    f = total_features / s
    return [max(2, int(round(c * f))) for c in base]


def slot_key(slot: int, ids: torch.Tensor) -> torch.Tensor:
    return ((slot + 1) << SLOT_SHIFT) + ids


@dataclass
class Batch:
    """A device batch in the engine's flat slot-major layout."""

    keys: torch.Tensor  # int64 [S*B] (slot-major; -1 = padding)
    lod: torch.Tensor  # int64 [S*(B+1)]
    dense: torch.Tensor  # float [B, 13]
    label: torch.Tensor  # float [B]
    cvm: torch.Tensor  # float [B, 2] = [show=1, click=label]
    B: int
    S: int

    def to(self, device, non_blocking=False) -> "Batch":
        return Batch(*(t.to(device, non_blocking=non_blocking) for t in
                       (self.keys, self.lod, self.dense, self.label, self.cvm)), self.B, self.S)

    def pin_memory(self) -> "Batch":
        return Batch(*(t.pin_memory() for t in (self.keys, self.lod, self.dense, self.label, self.cvm)), self.B,
                     self.S)


class CriteoSynth:
    def __init__(self, total_features: int = 1_000_000_000, alpha: float = 1.05, seed: int = 0,
                 device: str = "cpu", cardinalities: Optional[List[int]] = None):
        self.card = cardinalities or scaled_cardinalities(total_features)
        self.S = len(self.card)
        self.alpha = alpha
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.card_t = torch.tensor(self.card, dtype=torch.float64, device=self.device)

    @property
    def total_features(self) -> int:
        return sum(self.card)

    def sample_ids(self, B: int) -> torch.Tensor:
        """[S, B] int64 ids, power-law popularity (continuous Zipf inverse CDF)."""
        u = torch.rand(self.S, B, generator=self.gen, device=self.device, dtype=torch.float64)
        a = self.alpha
        n = self.card_t.unsqueeze(1)
        if abs(a - 1.0) < 1e-9:
            x = torch.pow(n + 1, u) - 1
        else:
            x = torch.pow((torch.pow(n + 1, 1 - a) - 1) * u + 1, 1 / (1 - a)) - 1
        ids = x.floor().clamp_(min=0)
        ids = torch.minimum(ids, n - 1).to(torch.int64)
        # scramble ids inside each slot so popular ids are not clustered
        return ids

    def batch(self, B: int) -> Batch:
        S = self.S
        ids = self.sample_ids(B)
        slots = torch.arange(S, device=self.device, dtype=torch.int64).unsqueeze(1)
        keys = ((slots + 1) << SLOT_SHIFT) + ids  # [S, B]
        # hidden logistic model: weight per key from its hash
        from ..ops.reference import mix64

        hk = mix64(keys)
        w = ((hk & 0xFFFF).to(torch.float32) / 65535.0 - 0.5) * 0.6
        dense_raw = torch.empty(B, NUM_DENSE, device=self.device).exponential_(generator=self.gen)
        dense = torch.log1p(dense_raw * 10)
        logit = w.sum(0) + 0.3 * (dense[:, 0] - 1.0) - 1.2
        label = (torch.rand(B, generator=self.gen, device=self.device) < torch.sigmoid(logit)).float()
        lod = (torch.arange(S, device=self.device).unsqueeze(1) * B
               + torch.arange(B + 1, device=self.device).unsqueeze(0)).reshape(-1).to(torch.int64)
        cvm = torch.stack([torch.ones_like(label), label], 1)
        return Batch(keys.reshape(-1).contiguous(), lod, dense.contiguous(), label, cvm, B, S)

    def all_keys_chunks(self, chunk: int = 1 << 26):
        """Yield every key of the feature space (for pre-populating tables)."""
        for s, c in enumerate(self.card):
            start = 0
            while start < c:
                n = min(chunk, c - start)
                ids = torch.arange(start, start + n, device=self.device, dtype=torch.int64)
                yield slot_key(s, ids)
                start += n


def ragged_batch(B: int, S: int, max_len: int, vocab: int, seed: int = 0, device="cpu",
                 empty_prob: float = 0.1) -> Batch:
    """Multi-key-per-slot synthetic batch (variable sequence lengths, empty
    slots allowed) for exercising the general LoD path."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    lens = torch.randint(0, max_len + 1, (S, B), generator=g)
    lens[torch.rand(S, B, generator=g) < empty_prob] = 0
    lod = torch.zeros(S, B + 1, dtype=torch.int64)
    flat = lens.reshape(-1).cumsum(0)
    starts = torch.cat([torch.zeros(1, dtype=torch.int64), flat[:-1]]).view(S, B)
    lod[:, :B] = starts
    lod[:, B] = starts[:, -1] + lens[:, -1]
    L = int(flat[-1])
    keys = torch.empty(L, dtype=torch.int64)
    slot_of = torch.repeat_interleave(torch.arange(S), lens.sum(1))
    ids = torch.randint(0, vocab, (L,), generator=g)
    keys = ((slot_of + 1) << SLOT_SHIFT) + ids
    label = (torch.rand(B, generator=g) < 0.3).float()
    dense = torch.rand(B, NUM_DENSE, generator=g)
    cvm = torch.stack([torch.ones(B), label], 1)
    return Batch(keys, lod.reshape(-1), dense, label, cvm, B, S).to(device)
