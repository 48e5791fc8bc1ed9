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

GPU tables are written by the native streaming saver (``GpuTable.save_stream``:
chunked device compaction -> pinned ring -> writer threads, bounded HBM);
feature-type codec tables (int16 / variable / SparseAdam) are decoded to their
canonical fp32 rows on the device in the same pass.  CPU tables and
PBX_SAVE_STREAM=0 use the export-based writer below.  Both produce the same
files.
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


# Streaming native saver (csrc/hip/ckpt.hip + ckpt_saver.cpp) for plain-
# layout GPU tables: the table is walked in chunks of this many row slots
# through two device buffers (2 x chunk x (8 + 4*stride) B of HBM, ~190 MB at
# the default) and pinned host buffers into writer threads -- no device copy
# of the table, no Python loop over rows.
STREAM_CHUNK_ROWS = int(os.environ.get("PBX_SAVE_CHUNK_ROWS", str(1 << 22)))
STREAM_THREADS = int(os.environ.get("PBX_SAVE_THREADS", str(min(16, os.cpu_count() or 4))))
last_save_stats: dict = {}


def _save_max_cols() -> int:
    from .. import _native

    return int(getattr(_native.hip(), "kSaveMaxCols", 192))


def _streamable(table) -> bool:
    t = getattr(table, "t", None)
    if t is None or not hasattr(t, "save_stream") or os.environ.get("PBX_SAVE_STREAM", "1") == "0":
        return False
    c = getattr(table, "codec", None)
    # the device-side decode map is a kernel argument of kSaveMaxCols entries:
    # wider canonical rows (e.g. SparseAdam at large dims) take the export path
    return c is None or int(c.canon_width) <= _save_max_cols()


def _tiered(table) -> bool:
    return hasattr(table, "save_tiers") and os.environ.get("PBX_SAVE_STREAM", "1") != "0"


def _decode_args(table):
    """(column map, scale, embedding width) of a codec table's canonical rows;
    an empty map = rows as stored."""
    c = getattr(table, "codec", None)
    if c is None:
        return [], 1.0, 0
    return c.save_map(), float(c.qscale), int(c.DX)


def _out_stride(table) -> int:
    c = getattr(table, "codec", None)
    return int(c.canon_width) if c is not None else int(table.t.stride)


def _stream(table, kind: int, mode: int, reset: bool, cfg: Optional[SaveConfig], nonclk: float, clk: float,
            keys_path: str, vals_path: str = "", collect: bool = False):
    cfg = cfg or SaveConfig()
    dmap, dscale, ddim = _decode_args(table)
    with torch.cuda.device(table.device):
        rows, chunks, gpu_s, write_s, total_s, keys = table.t.save_stream(
            kind, mode, reset, float(cfg.base_threshold), float(cfg.delta_threshold), float(cfg.delta_keep_days),
            float(nonclk), float(clk), float(cfg.embedx_threshold), keys_path, vals_path, STREAM_CHUNK_ROWS,
            STREAM_THREADS, collect, dmap, dscale, ddim)
    last_save_stats.clear()
    last_save_stats.update(rows=rows, chunks=chunks, gpu_s=gpu_s, write_s=write_s, total_s=total_s, native=True)
    return int(rows), keys


def _write_meta(path: str, dim: int, stride: int, date, world: Optional[int] = None):
    meta = {"format": FORMAT, "dim": dim, "stride": stride, "layout": row_layout(dim), "date": date}
    if world is not None:
        # parts written by `world` owner-sharded ranks: part r holds exactly the
        # keys that rank r of a same-sized job owns (load fast path)
        meta["world"] = int(world)
    with open(os.path.join(path, "meta.json"), "w") as f:
        json.dump(meta, f)


def save_batch_model(table, path: str, rank: int = 0, date: Optional[str] = None, world: Optional[int] = None) -> int:
    os.makedirs(path, exist_ok=True)
    if _tiered(table):  # host + SSD tiers, natively streamed
        n, _ = table.save_tiers(0, 0, False, None, 0.0, 0.0, os.path.join(path, f"part-{rank:05d}.keys.npy"),
                                os.path.join(path, f"part-{rank:05d}.vals.npy"))
        last_save_stats.clear()
        last_save_stats.update(table.last_save)
        if rank == 0:
            _write_meta(path, table.dim, int(table.stride), date, world)
        return n
    if _streamable(table):
        n, _ = _stream(table, 0, 0, False, None, 0.0, 0.0, os.path.join(path, f"part-{rank:05d}.keys.npy"),
                       os.path.join(path, f"part-{rank:05d}.vals.npy"))
        if rank == 0:
            _write_meta(path, table.dim, _out_stride(table), date, world)
        return n
    h, v = table.export(True)
    keys = ref.unmix64(h.cpu()).numpy().view(np.uint64)
    vals = v.float().cpu().numpy()
    np.save(os.path.join(path, f"part-{rank:05d}.keys.npy"), keys, allow_pickle=False)
    np.save(os.path.join(path, f"part-{rank:05d}.vals.npy"), vals, allow_pickle=False)
    if rank == 0:
        _write_meta(path, table.dim, int(vals.shape[1]) if vals.ndim == 2 else 0, date, world)
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


# Streaming load: parts are read in chunks of this many rows (positioned reads
# past the .npy header, no memory map: a mapping keeps every page it touched
# resident), so a rank's host RAM for a load stays at ~2 chunks whatever the
# model size (a 1e9-row model is ~90 GB of parts).
LOAD_CHUNK_ROWS = int(os.environ.get("PBX_LOAD_CHUNK_ROWS", str(1 << 22)))


def read_meta(path: str) -> dict:
    fn = os.path.join(path, "meta.json")
    if not os.path.exists(fn):
        return {}
    with open(fn) as f:
        return json.load(f)


def list_parts(path: str):
    """Part ids of a batch model directory, ascending."""
    return sorted(int(f[5:10]) for f in os.listdir(path) if f.startswith("part-") and f.endswith(".keys.npy"))


def _npy_layout(fn: str):
    """(shape, dtype, data offset) of a .npy file, from its header only
    (numpy.lib.format: no pickle is ever read; object arrays are refused)."""
    with open(fn, "rb") as f:
        version = np.lib.format.read_magic(f)
        if version == (1, 0):
            shape, fortran, dtype = np.lib.format.read_array_header_1_0(f)
        else:
            shape, fortran, dtype = np.lib.format.read_array_header_2_0(f)
        if fortran or dtype.hasobject:
            raise ValueError(f"{fn}: not a C-order plain array")
        return shape, dtype, f.tell()


def part_rows(path: str, part: int) -> int:
    return int(_npy_layout(os.path.join(path, f"part-{part:05d}.keys.npy"))[0][0])


def iter_part_chunks(path: str, part: int, chunk_rows: int):
    """(feasigns uint64 [n], rows f32 [n, stride]) chunks of one part, read
    with positioned reads of the raw array data: only the chunk being yielded
    is resident (and the page cache's copy, which the kernel may drop)."""
    kf = os.path.join(path, f"part-{part:05d}.keys.npy")
    vf = os.path.join(path, f"part-{part:05d}.vals.npy")
    (n,), kd, ko = _npy_layout(kf)
    vshape, vd, vo = _npy_layout(vf)
    if vshape[0] != n:
        raise ValueError(f"part {part}: {n} keys but {vshape[0]} value rows")
    width = int(np.prod(vshape[1:])) if len(vshape) > 1 else 1
    step = max(1, int(chunk_rows))
    with open(kf, "rb") as fk, open(vf, "rb") as fv:
        for a in range(0, n, step):
            b = min(n, a + step)
            fk.seek(ko + a * kd.itemsize)
            k = np.fromfile(fk, dtype=kd, count=b - a)
            fv.seek(vo + a * width * vd.itemsize)
            v = np.fromfile(fv, dtype=vd, count=(b - a) * width).reshape((b - a,) + tuple(vshape[1:]))
            try:  # the chunk is consumed: let the page cache drop it
                os.posix_fadvise(fk.fileno(), ko + a * kd.itemsize, (b - a) * kd.itemsize, os.POSIX_FADV_DONTNEED)
                os.posix_fadvise(fv.fileno(), vo + a * width * vd.itemsize, (b - a) * width * vd.itemsize,
                                 os.POSIX_FADV_DONTNEED)
            except (AttributeError, OSError):
                pass
            yield k.astype(np.uint64, copy=False), v.astype(np.float32, copy=False)


def save_xbox(table, path: str, mode: str, cfg: SaveConfig, nonclk: float, clk: float, rank: int = 0,
              on_reset=None, reset_live=None) -> int:
    """Write the xbox text model ('base' or 'delta'); resets delta_score of
    the saved rows (ctr_accessor.cc:121-124,153-162).  ``on_reset(h)`` is
    called with the saved mixed keys (another tier holding live copies of
    the rows applies the same reset); for the tiers ``reset_live(mode)``
    instead re-applies the save rule to the live copies (no key list)."""
    os.makedirs(path, exist_ok=True)
    # rows are canonical: a codec table's embedding block is embedx + expand
    codec = getattr(table, "codec", None)
    dim = int(codec.DX) if codec is not None else table.dim
    l = row_layout(dim)
    fn = os.path.join(path, f"part-{rank:05d}.txt")
    if _tiered(table):
        n, saved = table.save_tiers(1, 1 if mode == "base" else 2, True, cfg, nonclk, clk, fn,
                                    collect=on_reset is not None and reset_live is None)
        last_save_stats.clear()
        last_save_stats.update(table.last_save)
        if reset_live is not None:
            reset_live(mode)
        elif on_reset is not None and saved is not None and saved.numel():
            on_reset(saved)
        return n
    if _streamable(table):
        n, saved = _stream(table, 1, 1 if mode == "base" else 2, True, cfg, nonclk, clk, fn,
                           collect=on_reset is not None)
        if on_reset is not None and saved is not None and saved.numel():
            on_reset(saved.to(table.device))
        return n
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
