"""SSD tier of the HBM -> pinned host -> SSD embedding cache.

Log-structured segment store: every spill writes an immutable sorted segment
(``seg-NNNNNN.keys.npy`` + ``.vals.npy``); lookups binary-search segments
newest-first (values are memory-mapped, so only touched pages are read);
``compact()`` merges segments newest-wins and drops tombstoned keys.
BoxPS keeps its SSD tier inside the closed libbox_ps.so
(``LoadSSD2Mem``, ``box_wrapper.cc:1320-1324``); this is the open equivalent.
"""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np
import torch


class SsdStore:
    def __init__(self, path: str, stride: int):
        self.path = path
        self.stride = stride
        os.makedirs(path, exist_ok=True)
        self.segments: List[Tuple[np.ndarray, str]] = []
        self._next = 0
        for f in sorted(os.listdir(path)):
            if f.startswith("seg-") and f.endswith(".keys.npy"):
                keys = np.load(os.path.join(path, f), allow_pickle=False)
                self.segments.append((keys, os.path.join(path, f.replace(".keys.npy", ".vals.npy"))))
                self._next = max(self._next, int(f[4:10]) + 1)
        self.tombstones = set()

    def __len__(self):
        return int(sum(k.shape[0] for k, _ in self.segments))

    def put(self, h: torch.Tensor, v: torch.Tensor):
        if h.numel() == 0:
            return
        hk = h.cpu().numpy().astype(np.int64)
        order = np.argsort(hk, kind="stable")
        hk = hk[order]
        vv = v.float().cpu().numpy()[order]
        name = f"seg-{self._next:06d}"
        self._next += 1
        kp = os.path.join(self.path, name + ".keys.npy")
        vp = os.path.join(self.path, name + ".vals.npy")
        np.save(kp, hk, allow_pickle=False)
        np.save(vp, vv, allow_pickle=False)
        self.segments.append((hk, vp))
        for k in hk.tolist():
            self.tombstones.discard(k)

    def get(self, h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(found mask, values [n, stride]) -- newest segment wins."""
        q = h.cpu().numpy().astype(np.int64)
        n = q.shape[0]
        found = np.zeros(n, dtype=bool)
        out = np.zeros((n, self.stride), dtype=np.float32)
        for keys, vp in reversed(self.segments):
            if found.all() or keys.shape[0] == 0:
                continue
            pos = np.searchsorted(keys, q)
            pos_c = np.minimum(pos, keys.shape[0] - 1)
            hit = (~found) & (keys[pos_c] == q)
            if hit.any():
                vals = np.load(vp, mmap_mode="r", allow_pickle=False)
                out[hit] = vals[pos_c[hit]]
                found |= hit
        if self.tombstones:
            dead = np.array([k in self.tombstones for k in q.tolist()], dtype=bool)
            found &= ~dead
        return torch.from_numpy(found), torch.from_numpy(out)

    def delete(self, h: torch.Tensor):
        self.tombstones.update(h.cpu().numpy().astype(np.int64).tolist())

    def compact(self):
        if len(self.segments) <= 1 and not self.tombstones:
            return
        allk, allv = [], []
        for keys, vp in self.segments:
            allk.append(keys)
            allv.append(np.load(vp, allow_pickle=False))
        k = np.concatenate(allk) if allk else np.zeros(0, np.int64)
        v = np.concatenate(allv) if allv else np.zeros((0, self.stride), np.float32)
        # newest wins: reverse, unique keeps first occurrence
        k, v = k[::-1], v[::-1]
        uk, idx = np.unique(k, return_index=True)
        v = v[idx]
        if self.tombstones:
            live = ~np.isin(uk, np.array(sorted(self.tombstones), dtype=np.int64))
            uk, v = uk[live], v[live]
        for _, vp in self.segments:
            os.remove(vp)
            os.remove(vp.replace(".vals.npy", ".keys.npy"))
        self.segments = []
        self.tombstones = set()
        self.put(torch.from_numpy(uk), torch.from_numpy(np.ascontiguousarray(v)))
