"""Auxiliary BoxWrapper tables.

* :class:`GpuReplicaCache` -- small fully replicated per-GPU embedding table
  addressed by a dense offset (the data feed stores offsets as feasigns);
  ``pull_cache_value`` gathers rows.  Reference ``GpuReplicaCache``
  (``fw/fleet/box_wrapper.h:63-122``, kernel ``box_wrapper.cu:1210-1224``).
* :class:`InputTable` -- string key -> dense vector host table used by
  ``lookup_input`` (``box_wrapper.h:124-197``); the data feed maps keys to
  offsets, lookups gather on the host and copy to the device.
* :class:`ExpandEmbedding` -- the "expand" embedding of
  ``pull_box_extended_sparse`` (``ops/pull_box_extended_sparse_op.*``): a
  second sparse engine keyed by the same feasigns whose embedx holds the
  expand vector; pulled/pushed alongside the main records.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import reference as ref


class GpuReplicaCache:
    def __init__(self, dim: int, device=None):
        self.dim = int(dim)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._host: List[np.ndarray] = []
        self._n = 0
        self.table: Optional[torch.Tensor] = None

    def add_items(self, rows) -> int:
        """Append rows [n, dim]; returns the offset of the first one."""
        a = np.asarray(rows, dtype=np.float32).reshape(-1, self.dim)
        off = self._n
        self._host.append(a)
        self._n += a.shape[0]
        return off

    def load_native(self, store):
        """Rows a data feed appended to a native ReplicaStore during the load
        (replica-cache data feed; offsets are the instances' feasigns)."""
        data = store.data()
        self.dim = int(data.shape[1])  # a pass's cache takes the feed's row width
        self._host = [data.numpy()]
        self._n = data.shape[0]
        self.table = None
        return self

    def to_hbm(self):
        data = np.concatenate(self._host, 0) if self._host else np.zeros((0, self.dim), np.float32)
        self.table = torch.from_numpy(data).to(self.device)
        return self.table

    def pull(self, ids: torch.Tensor, size: int) -> torch.Tensor:
        if self.table is None:
            self.to_hbm()
        idx = ids.reshape(-1).to(self.table.device).long().clamp(0, max(self._n - 1, 0))
        out = self.table.index_select(0, idx)
        if size != self.dim:
            out = out[:, :size] if size < self.dim else torch.nn.functional.pad(out, (0, size - self.dim))
        return out

    def __len__(self):
        return self._n


class InputTable:
    """String key -> dense vector table for ``lookup_input``.  Backed by the
    native ``InputIndex`` (csrc/host/side_tables.cc) that the loader threads
    query while parsing (input-index data feed); lookups gather from an HBM
    copy of the rows (refreshed when rows were added) instead of a host
    gather + H2D per call."""

    def __init__(self, dim: int = 0):
        from .. import _native

        self.native = _native.host().InputIndex(int(dim)) if _native.host_available() else None
        self._py_index: Dict[str, int] = {}
        self._py_rows: List[np.ndarray] = []
        self.dim = int(dim)
        self._dev: Dict[str, torch.Tensor] = {}
        self._dev_n = -1

    def set_dim(self, dim: int):
        self.dim = int(dim)
        if self.native is not None and self.native.size() == 0:
            from .. import _native

            self.native = _native.host().InputIndex(self.dim)

    def add_index_data(self, key: str, vec) -> int:
        v = torch.as_tensor(np.asarray(vec, dtype=np.float32).reshape(-1))
        if self.native is not None:
            off = int(self.native.add(key, v))
            self.dim = int(self.native.dim())
            return off
        if self.dim == 0:
            self.dim = v.numel()
        if key not in self._py_index:
            self._py_index[key] = len(self._py_rows)
            self._py_rows.append(v.numpy()[: self.dim])
        return self._py_index[key]

    def load_text(self, path: str, threads: int = 4) -> int:
        if self.native is not None:
            n = int(self.native.load_text([path], threads))
            self.dim = int(self.native.dim())
            return n
        n = 0
        with open(path) as f:
            for line in f:
                t = line.split()
                if t:
                    self.add_index_data(t[0], [float(x) for x in t[1:]])
                    n += 1
        return n

    def get_offset(self, key: str) -> int:
        if self.native is not None:
            return int(self.native.offset(key))
        return self._py_index.get(key, -1)

    def size(self) -> int:
        return int(self.native.size()) if self.native is not None else len(self._py_rows)

    def rows(self) -> torch.Tensor:
        if self.native is not None:
            return self.native.data()
        return torch.from_numpy(np.stack(self._py_rows, 0)) if self._py_rows else torch.zeros(0, max(self.dim, 1))

    def lookup(self, ids: torch.Tensor, size: int, device) -> torch.Tensor:
        device = torch.device(device)
        n = self.size()
        key = str(device)
        if self._dev_n != n or key not in self._dev:
            self._dev = {key: self.rows().to(device)}
            self._dev_n = n
        data = self._dev[key]
        idx = ids.reshape(-1).to(device).long()
        ok = (idx >= 0) & (idx < data.shape[0])
        rows = data.index_select(0, idx.clamp(0, max(data.shape[0] - 1, 0))) if data.shape[0] else \
            torch.zeros(idx.numel(), max(self.dim, 1), device=device)
        rows = rows * ok.unsqueeze(1).to(rows.dtype)
        w = min(size, rows.shape[1])
        out = torch.zeros(idx.numel(), size, device=device)
        out[:, :w] = rows[:, :w]
        return out


class _PullExtended(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, keys, lod, main, ext, B, S, emb_size, ext_size, bs_scale):
        recs, st = main.pull_records(keys, lod, B, S)
        erecs, est = ext.pull_records(keys, lod, B, S)
        ctx.main, ctx.ext, ctx.st, ctx.est, ctx.bs = main, ext, st, est, bs_scale
        ctx.emb_size, ctx.ext_size, ctx.E = emb_size, ext_size, recs.shape[1]
        out = recs[:, :emb_size] if emb_size <= recs.shape[1] else torch.nn.functional.pad(
            recs, (0, emb_size - recs.shape[1]))
        ex = erecs[:, 3:3 + ext_size]
        return out.contiguous(), ex.contiguous()

    @staticmethod
    def backward(ctx, g, gex):
        E = ctx.E
        gm = torch.zeros(g.shape[0], E, device=g.device, dtype=torch.float32)
        w = min(E, g.shape[1])
        gm[:, :w] = g[:, :w].float()
        ctx.main.push_records(ctx.st, gm, 2, ctx.bs)
        if gex is not None:
            ge = torch.zeros(gex.shape[0], 3 + ctx.ext.dim, device=gex.device, dtype=torch.float32)
            ge[:, :2] = gm[:, :2]  # same show/click statistics drive the expand rows
            ge[:, 3:3 + gex.shape[1]] = gex.float()
            ctx.ext.push_records(ctx.est, ge, 2, ctx.bs)
        return (None,) * 10


class _PullExtendedCodec(torch.autograd.Function):
    """pull_box_extended_sparse on one engine whose rows carry the expand
    block (feature codec with De > 0, csrc/hip/feature_ops.hip): one pull
    returns [show, click, embed_w, embedx[D], expand[De]] per occurrence and
    one push updates both blocks."""

    @staticmethod
    def forward(ctx, anchor, keys, lod, eng, B, S, emb_size, ext_size, bs_scale):
        recs, st = eng.pull_records(keys, lod, B, S, with_expand=True)
        E = 3 + eng.dim
        ctx.eng, ctx.st, ctx.bs, ctx.E, ctx.W = eng, st, bs_scale, E, recs.shape[1]
        out = recs[:, :min(emb_size, E)]
        if emb_size > E:
            out = torch.nn.functional.pad(out, (0, emb_size - E))
        ex = recs[:, E:E + ext_size]
        return out.contiguous(), ex.contiguous()

    @staticmethod
    def backward(ctx, g, gex):
        gm = torch.zeros(ctx.st.L, ctx.W, device=ctx.st.lod.device, dtype=torch.float32)
        if g is not None:
            w = min(ctx.E, g.shape[1])
            gm[:, :w] = g[:, :w].float()
        if gex is not None:
            gm[:, ctx.E:ctx.E + gex.shape[1]] = gex.float()
        ctx.eng.push_records(ctx.st, gm, 2, ctx.bs)
        return (None,) * 9


class _PullExtendedVar(torch.autograd.Function):
    """pull_box_extended_sparse with the variable feature type (codec kind
    3): every feature has its own embedding size (D or De, set at creation
    by the slot it was created from).  Each slot is pulled into ONE output:
    the expand output when the slot has one (mask bit 1), else the embedx
    output; columns past the feature's size read as zero.  The push takes
    the cvm / embed_w gradients from that output and the embedding gradients
    only when the feature's size matches the output (reference
    PullCopyVariable / PushMergeCopyVariable, box_wrapper.cu:271-322,
    714-875, total_dims bit 0 = size D, bit 1 = size De)."""

    @staticmethod
    def forward(ctx, anchor, keys, lod, eng, B, S, emb_size, ext_size, bs_scale, route):
        recs, st = eng.pull_records(keys, lod, B, S, with_expand=True)
        c = eng.codec
        DX = c.DX
        xs = recs[:, 3 + DX]
        slot_of_occ, _ = ref.occurrence_map(lod.cpu(), S, B)
        slot_of_occ = slot_of_occ.to(keys.device)
        to_ex = route.to(keys.device)[slot_of_occ.long()]
        ctx.eng, ctx.st, ctx.bs, ctx.DX = eng, st, bs_scale, DX
        ctx.save_for_backward(xs, to_ex, slot_of_occ)

        def cols(n):
            out = recs[:, :min(n, 3 + DX)]
            return torch.nn.functional.pad(out, (0, n - out.shape[1])) if n > out.shape[1] else out

        out = cols(emb_size).clone()
        ex = cols(ext_size).clone()
        # a slot writes only its own output (the other one stays zero)
        out[to_ex] = 0
        ex[~to_ex] = 0
        # embedding columns beyond the output's dim: embedx output shows D
        if emb_size > 3 + c.D:
            out[:, 3 + c.D:] = 0
        return out, ex

    @staticmethod
    def backward(ctx, g, gex):
        xs, to_ex, slot_of_occ = ctx.saved_tensors
        c = ctx.eng.codec
        L = ctx.st.L
        gm = torch.zeros(L, 3 + ctx.DX, device=xs.device, dtype=torch.float32)
        if g is None:
            g = torch.zeros(L, 3, device=xs.device)
        if gex is None:
            gex = torch.zeros(L, 3, device=xs.device)
        g, gex = g.float(), gex.float()
        head_x = torch.nn.functional.pad(g[:, :3], (0, max(0, 3 - g.shape[1])))
        head_e = torch.nn.functional.pad(gex[:, :3], (0, max(0, 3 - gex.shape[1])))
        gm[:, :3] = torch.where(to_ex.unsqueeze(1), head_e, head_x)
        we = min(c.De, gex.shape[1] - 3)
        wx = min(c.D, g.shape[1] - 3)
        if we > 0:
            sel = to_ex & (xs == c.De)
            gm[sel, 3:3 + we] = gex[sel, 3:3 + we]
        if wx > 0:
            sel = (~to_ex) & (xs == c.D)
            gm[sel, 3:3 + wx] = g[sel, 3:3 + wx]
        ctx.eng.push_records(ctx.st, gm, 2, ctx.bs, slot_of_occ)
        return (None,) * 10


def pull_extended_var(eng, keys, lod, B, S, emb_size: int, ext_size: int, mask=None):
    """Variable feature type pull (see _PullExtendedVar).  mask[s] as in
    _pull_box_extended_sparse: bit 1 = slot s has an expand output."""
    from ..ops.sparse import _anchor

    mask = list(mask) if mask else [3] * S
    route = torch.tensor([bool(m & 2) for m in mask[:S]] + [False] * max(0, S - len(mask)), dtype=torch.bool)
    ids = tuple(int(x) for x, r in zip(eng._slot_ids(S)[:S].tolist(), route.tolist()) if r)
    if getattr(eng.codec, "_vslot_ids", None) != sorted(set(ids)):
        eng.codec.set_expand_slots(ids)
    return _PullExtendedVar.apply(_anchor(keys.device), keys, lod, eng, B, S, emb_size, ext_size, float(B), route)


def pull_extended_codec(eng, keys, lod, B, S, emb_size: int, ext_size: int):
    from ..ops.sparse import _anchor

    return _PullExtendedCodec.apply(_anchor(keys.device), keys, lod, eng, B, S, emb_size, ext_size, float(B))


class ExpandEmbedding:
    """Expand-embedding companion engine (same keys, embedx = expand vector)."""

    def __init__(self, main_engine, expand_dim: int):
        from .config import PSConfig
        from .sparse_engine import SparseEngine

        cfg = PSConfig(embedx_dim=int(expand_dim))
        cfg.sgd = main_engine.cfg.sgd
        self.engine = SparseEngine(cfg, main_engine.max_keys, main_engine.device,
                                   capacity=getattr(main_engine.table, "capacity", 1 << 20),
                                   group=main_engine.group, auto_insert=True, comm=main_engine.comm)
        self.main = main_engine

    def register_keys(self, keys: torch.Tensor):
        self.engine.register_keys(keys)

    def pull(self, keys, lod, B, S, emb_size, ext_size) -> Tuple[torch.Tensor, torch.Tensor]:
        from ..ops.sparse import _anchor

        return _PullExtended.apply(_anchor(keys.device), keys, lod, self.main, self.engine, B, S, emb_size,
                                   ext_size, float(B))
