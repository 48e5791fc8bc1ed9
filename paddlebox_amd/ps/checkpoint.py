"""Sparse model checkpoints: batch model (full training state) + xbox serving
model (base / delta), BoxPS layout.

The real BoxPS save format lives inside the closed libbox_ps.so
(``SaveBase/SaveDelta`` call sites ``box_wrapper.cc:1286-1318``); the
semantics reproduced here are the PSCore CTR accessor's
(``distributed/ps/table/ctr_accessor.cc:102-170,310-341``):

* batch model  -- every feature, full value row (optimizer state included);
  binary ``.npy`` (loaded with ``allow_pickle=False``).
* xbox base    -- features with score >= base_threshold and
  unseen_days <= delta_keep_days; saving resets delta_score.
* xbox delta   -- additionally delta_score >= delta_threshold; resets it.
* xbox text    -- ``feasign \t slot unseen_days delta_score show click embed_w
  embed_g2sum [embedx_w... embedx_g2sum]``; embedx only when
  score >= embedx_threshold.

Layout: ``<path>/part-<rank>.keys.npy``, ``.vals.npy``, ``meta.json``;
xbox ``<path>/part-<rank>.txt``.
"""
from __future__ import annotations

import json
import os
from typing import Optional, Tuple

import numpy as np
import torch

from ..ops import reference as ref
from .config import SaveConfig, row_layout

FORMAT = "pbx-batch-model-v1"


def _score(v: torch.Tensor, nonclk: float, clk: float) -> torch.Tensor:
    return (v[:, 0] - v[:, 1]) * nonclk + v[:, 1] * clk


def select_rows(h: torch.Tensor, v: torch.Tensor, dim: int, mode: str, cfg: SaveConfig, nonclk: float,
                clk: float) -> torch.Tensor:
    """Boolean mask of rows saved for mode in {'all', 'base', 'delta'}."""
    l = row_layout(dim)
    if mode == "all":
        return torch.ones(h.numel(), dtype=torch.bool, device=h.device)
    keep = (_score(v, nonclk, clk) >= cfg.base_threshold) & (v[:, l["unseen_days"]] <= cfg.delta_keep_days)
    if mode == "delta":
        keep &= v[:, l["delta_score"]] >= cfg.delta_threshold
    return keep


def save_batch_model(table, path: str, rank: int = 0, date: Optional[str] = None) -> int:
    os.makedirs(path, exist_ok=True)
    h, v = table.export(True)
    keys = ref.unmix64(h.cpu()).numpy().view(np.uint64)
    vals = v.float().cpu().numpy()
    np.save(os.path.join(path, f"part-{rank:05d}.keys.npy"), keys, allow_pickle=False)
    np.save(os.path.join(path, f"part-{rank:05d}.vals.npy"), vals, allow_pickle=False)
    if rank == 0:
        meta = {"format": FORMAT, "dim": table.dim, "stride": int(vals.shape[1]) if vals.ndim == 2 else 0,
                "layout": row_layout(table.dim), "date": date}
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f)
    return int(keys.shape[0])


def load_batch_model_parts(path: str, rank: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Read all (or one rank's) parts: (feasigns uint64, value rows f32)."""
    files = sorted(f for f in os.listdir(path) if f.endswith(".keys.npy"))
    if rank is not None:
        files = [f for f in files if f == f"part-{rank:05d}.keys.npy"]
    ks, vs = [], []
    for f in files:
        ks.append(np.load(os.path.join(path, f), allow_pickle=False))
        vs.append(np.load(os.path.join(path, f.replace(".keys.npy", ".vals.npy")), allow_pickle=False))
    if not ks:
        return np.zeros(0, np.uint64), np.zeros((0, 0), np.float32)
    return np.concatenate(ks), np.concatenate(vs)


def save_xbox(table, path: str, mode: str, cfg: SaveConfig, nonclk: float, clk: float, rank: int = 0,
              on_reset=None) -> int:
    """Write the xbox text model ('base' or 'delta'); resets delta_score of
    the saved rows (ctr_accessor.cc:121-124,153-162).  ``on_reset(h)`` is
    called with the saved mixed keys (another tier holding live copies of
    the rows applies the same reset)."""
    os.makedirs(path, exist_ok=True)
    dim = table.dim
    l = row_layout(dim)
    h, v = table.export(True)
    keep = select_rows(h, v, dim, mode, cfg, nonclk, clk)
    hk, vk = h[keep], v[keep]
    # reset delta score of saved rows
    if hk.numel():
        vr = vk.clone()
        vr[:, l["delta_score"]] = 0
        table.assign(hk, vr)
        if on_reset is not None:
            on_reset(hk)
    keys = ref.unmix64(hk.cpu()).numpy().view(np.uint64)
    vv = vk.float().cpu().numpy()
    with_x = (_score(vk, nonclk, clk) >= cfg.embedx_threshold).cpu().numpy()
    fn = os.path.join(path, f"part-{rank:05d}.txt")
    with open(fn, "w") as f:
        for i in range(keys.shape[0]):
            row = vv[i]
            head = [row[l["slot"]], row[l["unseen_days"]], row[l["delta_score"]], row[0], row[1], row[2],
                    row[l["embed_g2sum"]]]
            if with_x[i] and row[l["mf_size"]] != 0:
                head += list(row[3:3 + dim]) + [row[l["embedx_g2sum"]]]
            f.write(f"{int(keys[i])}\t" + " ".join(f"{x:.6g}" for x in head) + "\n")
    return int(keys.shape[0])


def load_xbox_text(fn: str, dim: int):
    """Parse an xbox text part back to (feasigns, value rows)."""
    l = row_layout(dim)
    ks, rows = [], []
    with open(fn) as f:
        for line in f:
            k, rest = line.rstrip("\n").split("\t")
            x = [float(t) for t in rest.split()]
            v = np.zeros(l["stride"], np.float32)
            v[l["slot"]], v[l["unseen_days"]], v[l["delta_score"]] = x[0], x[1], x[2]
            v[0], v[1], v[2], v[l["embed_g2sum"]] = x[3], x[4], x[5], x[6]
            if len(x) > 7:
                v[3:3 + dim] = x[7:7 + dim]
                v[l["embedx_g2sum"]] = x[7 + dim]
                v[l["mf_size"]] = 1
            ks.append(int(k))
            rows.append(v)
    return np.array(ks, dtype=np.uint64), (np.stack(rows) if rows else np.zeros((0, l["stride"]), np.float32))


def write_manifest(root: str, **kw):
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "manifest.json"), "w") as f:
        json.dump(kw, f, indent=1, sort_keys=True)
