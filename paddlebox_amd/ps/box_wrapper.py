"""BoxWrapper: the BoxPS facade (singleton) -- pass lifecycle, feature table,
tiers, checkpoints, metrics, phases, timers.

Reference contract: ``fw/fleet/box_wrapper.{h,cc}`` (SetInstance :651-684,
pass lifecycle :120-210, model IO :1201-1324, metrics :916-1083, timers
:1085-1138) and the closed BoxPS API enumerated in SURVEY §2.1.

Process model (MI355X-first): one process per GPU; this object is the
per-process instance.  The feature table is sharded over the ranks of the
process group by ``owner_of(mix64(key))``; key/value exchange is all-to-all
over RCCL (see ``sparse_engine``).

Tiers:
  * ``hbm`` (default): the GPU table holds the whole shard (288 GB HBM3E per
    MI355X holds ~3.5e9 8-dim features); feed pass inserts new keys.
  * ``tiered``: the host table (native C++ CpuTable) is authoritative; each
    pass stages its working set into HBM at EndFeedPass and writes it back at
    EndPass; cold host rows spill to the SSD segment store.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from ..metrics.registry import MetricRegistry
from ..ops import reference as ref
from ..utils import flags as _flags
from ..utils.dayid import make_day_id_str
from ..utils.log import logger
from ..utils.timer import StageTimers
from .. import _native
from . import checkpoint as ckpt
from .config import PSConfig, feature_pull_offsets, feature_push_offsets, row_layout
from .cpu_table import CpuSparseTable
from .sparse_engine import SparseEngine


class PSAgent:
    """Feed-pass key collector (boxps::PSAgentBase AddKey/AddKeys,
    box_wrapper.cc:1185-1200).  ``native`` is the sharded C++ key set the
    dataset's loader threads register parsed feasigns into while a feed pass
    is open (csrc/host/key_agent.cc); keys added from Python (device tensors
    included) are merged at ``keys()``."""

    def __init__(self, n_threads: int = 30):
        self.n = n_threads
        self._parts: List[List[torch.Tensor]] = [[] for _ in range(n_threads)]
        self._lock = threading.Lock()
        self.native = _native.host().KeyAgent(64) if _native.host_available() else None

    def add_key(self, key: int, tid: int = 0):
        self._parts[tid % self.n].append(torch.tensor([key], dtype=torch.int64))

    def add_keys(self, keys: torch.Tensor, tid: int = 0):
        # kept where they are: device keys are deduplicated on the device
        self._parts[tid % self.n].append(keys.reshape(-1).to(torch.int64))

    def keys(self) -> torch.Tensor:
        allk = [t for p in self._parts for t in p]
        nat = self.native.keys() if self.native is not None and self.native.size() else None
        if nat is not None:
            if not allk:
                return nat  # unique already, padding keys excluded
            allk.append(nat)
        if not allk:
            return torch.empty(0, dtype=torch.int64)
        dev = next((t.device for t in allk if t.is_cuda), allk[0].device)
        k = torch.cat([t.to(dev) for t in allk])
        k = k[(k != 0) & (k != -1)]
        return torch.unique(k)


class BoxWrapper:
    _instance: Optional["BoxWrapper"] = None

    def __init__(self, embedx_dim: int = 8, expand_embed_dim: int = 0, feature_type: int = 0,
                 pull_embedx_scale: float = 1.0, device=None, group=None, cfg: Optional[PSConfig] = None):
        self.cfg = cfg or PSConfig(embedx_dim=embedx_dim, expand_embed_dim=expand_embed_dim,
                                   feature_type=feature_type, pull_embedx_scale=pull_embedx_scale)
        self.group = group
        ready = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if ready else 1
        self.rank = dist.get_rank(group) if ready else 0
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.engine: Optional[SparseEngine] = None
        self.slot_vector: List[int] = []
        self.slot_omit: List[int] = []
        self.lr_map: Dict[str, float] = {}
        self.metrics = MetricRegistry(group)
        self.timers = StageTimers(self.device)
        self.mode = "hbm"
        self.use_afs_api = False  # init_afs_api configured the remote file client
        self.host: Optional[CpuSparseTable] = None
        self.ssd = None  # tiered.SsdTier
        self.day_id = None
        self.pass_id = 0
        self.in_pass = False
        self.test_mode = False
        self.dataset_name = ""
        self.input_table_dim = 0
        self._agent: Optional[PSAgent] = None
        self._pass_keys: Optional[torch.Tensor] = None
        self.max_keys = 1 << 20
        self.capacity = 1 << 22
        self._replica = None
        self._input_table = None
        self._expand = None
        self.tier = None  # TieredStore (GPU tiered mode)
        # AucRunner (slot-importance evaluation); None = train/test mode
        self.auc_runner = None
        BoxWrapper._instance = self

    # ---------------------------------------------------------------- instance
    @staticmethod
    def set_instance(*a, **k) -> "BoxWrapper":
        return BoxWrapper(*a, **k)

    @staticmethod
    def get_instance() -> "BoxWrapper":
        if BoxWrapper._instance is None:
            raise RuntimeError("BoxWrapper not initialised")
        return BoxWrapper._instance

    # ---------------------------------------------------------------- init
    def initialize_gpu_and_load_model(self, conf_file: str = "", slot_vector: Sequence[int] = (),
                                      slot_omit_in_feedpass: Sequence[int] = (), model_path: str = "",
                                      lr_map: Optional[Dict[str, float]] = None, max_keys: Optional[int] = None,
                                      capacity: Optional[int] = None, mode: Optional[str] = None,
                                      ssd_path: Optional[str] = None, auto_insert: bool = False):
        """Parse the PS config, bind the device, register slots, load a base
        model (box_wrapper.cc:1201-1242)."""
        if conf_file and os.path.exists(conf_file):
            loaded = PSConfig.load(conf_file)
            loaded.embedx_dim = self.cfg.embedx_dim
            self.cfg = loaded
        self.slot_vector = list(slot_vector)
        self.slot_omit = list(slot_omit_in_feedpass)
        self.lr_map = dict(lr_map or {})
        mk = _flags.get_int("padbox_max_keys_per_batch")
        self.max_keys = int(max_keys or mk or self.max_keys)
        self.capacity = int(capacity or self.cfg.tier.hbm_capacity or self.capacity)
        self.mode = mode or ("tiered" if (ssd_path or self.cfg.tier.ssd_path) else "hbm")
        self.engine = SparseEngine(self.cfg, self.max_keys, self.device, capacity=self.capacity,
                                   slot_ids=[float(s) for s in self.slot_vector] or None, group=self.group,
                                   auto_insert=auto_insert)
        if self.mode == "tiered":
            from .tiered import HostTable, SsdTier, TieredStore

            codec = getattr(self.engine, "codec", None)
            # feature-type codecs: the host / SSD tiers keep the canonical fp32
            # rows the GPU table exports (re-encoded when staged back)
            self.host = (HostTable(codec.DX, stride=codec.canon_width) if codec is not None
                         else HostTable(self.cfg.embedx_dim))
            p = ssd_path or self.cfg.tier.ssd_path
            if p:
                self.ssd = SsdTier(os.path.join(p, f"rank{self.rank:05d}"), self.host.stride)
            if self.device.type == "cuda":
                self.tier = TieredStore(self.engine, self.host, self.ssd, self.cfg.sgd,
                                        spill_unseen=self.cfg.tier.spill_unseen_days,
                                        host_cap_rows=self.cfg.tier.ssd_spill_threshold)
        if model_path:
            self.load_model(model_path)
        return 0

    def set_slot_vector(self, slots: Sequence[int]):
        self.slot_vector = list(slots)
        if self.engine is not None:
            self.engine.set_slot_ids([float(s) for s in slots])

    # ---------------------------------------------------------------- feature layout
    def get_feature_pull_offsets(self):
        return feature_pull_offsets(self.cfg.embedx_dim, self.cfg.expand_embed_dim)

    def get_feature_push_offsets(self):
        return feature_push_offsets(self.cfg.embedx_dim, self.cfg.expand_embed_dim)

    @property
    def cvm_offset(self) -> int:
        return self.get_feature_pull_offsets()["cvm_offset"]

    # ---------------------------------------------------------------- feed pass
    def begin_feed_pass(self, date: Optional[str] = None) -> PSAgent:
        if date is not None:
            self.day_id = make_day_id_str(date)
        self._agent = PSAgent()
        return self._agent

    def end_feed_pass(self, agent: Optional[PSAgent] = None):
        agent = agent or self._agent
        keys = agent.keys() if agent is not None else torch.empty(0, dtype=torch.int64)
        with self.timers.span("feed_pass"):
            self._stage_keys(keys)
        self._agent = None

    def feed_pass(self, dataset_or_keys, date: Optional[str] = None):
        """FeedPass(date, keys) (deprecated form) / BoxHelper::ReadData2Memory."""
        agent = self.begin_feed_pass(date)
        if isinstance(dataset_or_keys, torch.Tensor):
            agent.add_keys(dataset_or_keys)
        else:
            agent.add_keys(dataset_or_keys.collect_keys())
            if self.auc_runner is not None:
                # GetRandomReplace + AddReplaceFeasign: the replacement
                # candidates' feasigns join this pass's working set
                agent.add_keys(self.auc_runner.prepare(dataset_or_keys))
        self.end_feed_pass(agent)

    # ---------------------------------------------------------------- AucRunner
    def initialize_auc_runner(self, slot_eval: Sequence[Sequence[str]], thread_num: int = 4, pool_size: int = 10000,
                              slot_list: Sequence[str] = ()):
        """InitializeAucRunner (box_wrapper.h:908-946): evaluation mode over
        ``len(slot_eval)`` phases; ``slot_eval[i]`` is a group of slot names
        whose feasigns get replaced by random other instances' ones."""
        from .auc_runner import AucRunner

        self.auc_runner = AucRunner(slot_eval, thread_num, pool_size)
        return self.auc_runner

    def auc_runner_mode(self) -> int:
        return 1 if self.auc_runner is not None else 0

    def _route(self, h: torch.Tensor) -> torch.Tensor:
        """Send mixed keys to their owner rank; returns this rank's keys."""
        if self.world == 1:
            return torch.unique(h)
        dev = self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        h = h.to(dev)
        owner = ref.owner_of(h, self.world)
        order = torch.argsort(owner, stable=True)
        h = h[order]
        counts = torch.bincount(owner, minlength=self.world)
        rc = torch.empty_like(counts)
        dist.all_to_all_single(rc, counts, group=self.group)
        recv = torch.empty(int(rc.sum()), dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv, h, rc.tolist(), counts.tolist(), group=self.group)
        return torch.unique(recv)

    def _stage_keys(self, keys: torch.Tensor):
        eng = self._require_engine()
        h = self._route(ref.mix64(keys.to(self.device if self.device.type == "cuda" else "cpu")))
        h = h.to(eng.device)
        if self._expand is not None:
            self._expand.engine.insert_local_mixed(h.to(self._expand.engine.device))
        if self.mode == "hbm":
            eng.insert_local_mixed(h)
            return
        if self.tier is not None:
            # staged into the second GPU table in the background; made live
            # by begin_pass (overlaps the current pass's training)
            self.tier.stage(h)
            return
        # tiered (CPU engine): host is authoritative
        hc = h.cpu()
        rows = self.host.probe(hc)
        miss = rows < 0
        if bool(miss.any()) and self.ssd is not None:
            found, vals = self.ssd.get(hc[miss])
            if bool(found.any()):
                mk = hc[miss][found]
                self.host.insert_mixed(mk, self.cfg.sgd)
                self.host.assign(mk, vals[found])
                self.ssd.delete(mk)
        self.host.insert_mixed(hc, self.cfg.sgd)
        vals = self.host.read(hc)
        self._pass_keys = hc
        eng.table.clear()
        eng.insert_local_mixed(h)
        eng.table.assign(h, vals.to(eng.device))

    # ---------------------------------------------------------------- pass
    def begin_pass(self):
        if self.tier is not None:
            with self.timers.span("begin_pass_activate"):
                self.tier.activate()
        self.in_pass = True
        self.pass_id += 1

    def end_pass(self, need_save_delta: bool = False):
        """EndPass: write back the working set (tiered), check exchange
        overflow, optional forced HBM release (box_wrapper.cc:186-210)."""
        eng = self._require_engine()
        if eng.check_overflow():
            raise RuntimeError("sparse key exchange overflowed its per-peer capacity this pass; "
                               "raise SparseEngine cap_factor (or leave it unset: worst-case slots never overflow)")
        if self.tier is not None:
            # export now, D2H + host scatter + SSD spill in the background
            with self.timers.span("end_pass_writeback"):
                self.tier.writeback()
        elif self.mode == "tiered":
            with self.timers.span("end_pass_writeback"):
                h, v = eng.table.export(True)
                self.host.assign(h.cpu(), v.cpu())
                self.host.stamp_keys(h.cpu(), self.pass_id)
                if self.ssd is not None:
                    self._spill_cold()
                    cap = int(self.cfg.tier.ssd_spill_threshold)
                    if cap > 0:
                        ck, cv = self.host._native.spill_oldest(cap)
                        self.ssd.put(ck, cv)
        if _flags.get_bool("enable_force_hbm_recyle") and self.device.type == "cuda":
            torch.cuda.empty_cache()
        if _flags.get_bool("enable_force_mem_recyle"):
            # release freed host memory back to the OS at the pass boundary
            import ctypes
            import gc

            gc.collect()
            try:
                ctypes.CDLL("libc.so.6").malloc_trim(0)
            except OSError:
                pass
        self.in_pass = False

    def _spill_cold(self, unseen_threshold: float = 1.0):
        from .config import row_layout

        h, v = self.host.export(True)
        if h.numel() == 0:
            return
        l = row_layout(self.cfg.embedx_dim)
        cold = v[:, l["unseen_days"]] >= unseen_threshold
        if bool(cold.any()):
            self.ssd.put(h[cold], v[cold])
            self.host._native.erase(h[cold].contiguous()) if self.host._native is not None else None

    def set_test_mode(self, is_test: bool):
        self.test_mode = bool(is_test)
        if self.engine is not None:
            self.engine.test_mode = self.test_mode

    # ---------------------------------------------------------------- model IO
    def _authoritative(self):
        """The table model IO and shrink act on: the GPU table (hbm), or in
        tiered mode the host + SSD tiers as one table (``TierView``: every
        feature, cold SSD rows included), made current first."""
        if self.mode == "tiered":
            self._sync_tiers()
            from .tiered import TierView

            v = getattr(self, "_tier_view", None)
            if v is None or v.host is not self.host or v.ssd is not self.ssd:
                v = self._tier_view = TierView(self.host, self.ssd)
            return v
        return self._require_engine().table

    def _sync_tiers(self):
        """Host tier current: finish the background write-back and, inside a
        pass, write the live GPU rows back synchronously first."""
        if self.tier is not None:
            # a next-pass staging still running moves SSD rows into the host
            # tier (host insert, then SSD delete) without the caller holding
            # the tier lock: a save / shrink walking the tiers meanwhile could
            # miss such a row or see it twice
            self.tier.wait_stage()
            self.tier.wait_writeback()  # also settles tier.retained
            if self.in_pass or self.tier.retained:
                self.tier.flush()
        elif self.mode == "tiered" and self.engine is not None and self.in_pass:
            h, v = self.engine.table.export(True)
            self.host.assign(h.cpu(), v.cpu())

    def _live_tables(self):
        """GPU tables holding live copies of tier rows: in a pass the live
        table; between passes with the GPU tier also the staged next pass
        (its activation carries live rows into the next pass)."""
        if self.mode != "tiered" or self.engine is None:
            return []
        if self.tier is not None:
            return self.tier.staged_tables()
        return [self.engine.table] if self.in_pass else []

    def _reset_delta_live(self, mode: str):
        """save_xbox reset delta_score of the saved rows in the host / SSD
        tiers; the live GPU rows must see the reset too, or a later write-back
        would restore the old scores.  Decided on the GPU rows themselves (the
        live ones were flushed into the host tier just before the save, so the
        save rule gives the same answer on both; a staged row the live table
        lacks is the host row) -- no per-saved-key list crosses host memory or
        the bus, whatever the size of the host + SSD model."""
        sg = self.cfg.sgd
        dcol = row_layout(self.cfg.embedx_dim)["delta_score"]
        for t in self._live_tables():
            if t.size() == 0:
                continue
            h, v = t.export(True)
            keep = ckpt.select_rows(h, v, self.cfg.embedx_dim, mode, self.cfg.save, sg.nonclk_coeff, sg.clk_coeff)
            if bool(keep.any()):
                vk = v[keep].clone()
                vk[:, dcol] = 0
                t.assign(h[keep], vk)

    def _push_live(self, h: torch.Tensor, v: torch.Tensor):
        """A tiered load / merge wrote rows into the host tier: GPU tables
        holding live copies of those keys take the loaded rows too (else the
        next activation or write-back brings the pre-load values back)."""
        for t in self._live_tables():
            hd = h.to(t.device)
            rows = t.probe(hd)
            ok = rows >= 0
            if bool(ok.any()):
                t.assign(hd[ok], v.to(t.device)[ok])

    def save_base(self, batch_model_path: str, xbox_model_path: str, date: str = "") -> str:
        """Full batch model + xbox base (box_wrapper.cc:1286-1305)."""
        t = self._authoritative()
        n = ckpt.save_batch_model(t, batch_model_path, self.rank, date, world=self.world)
        sg = self.cfg.sgd
        x = ckpt.save_xbox(t, xbox_model_path, "base", self.cfg.save, sg.nonclk_coeff, sg.clk_coeff, self.rank,
                           reset_live=self._reset_delta_live if self.mode == "tiered" else None)
        if self.rank == 0:
            ckpt.write_manifest(os.path.dirname(os.path.abspath(batch_model_path)) or ".", date=date,
                                pass_id=self.pass_id, embedx_dim=self.cfg.embedx_dim, world=self.world,
                                batch_model=batch_model_path, xbox=xbox_model_path, mode=self.mode,
                                flags=_flags.all_flags())
        return f"{batch_model_path} batch={n} xbox_base={x}"

    def save_delta(self, xbox_model_path: str) -> str:
        t = self._authoritative()
        sg = self.cfg.sgd
        x = ckpt.save_xbox(t, xbox_model_path, "delta", self.cfg.save, sg.nonclk_coeff, sg.clk_coeff, self.rank,
                           reset_live=self._reset_delta_live if self.mode == "tiered" else None)
        return f"{xbox_model_path} xbox_delta={x}"

    def load_model(self, model_path: str, merge: bool = False, update_type: str = "add", model_index: int = 0):
        """Load a batch model, streamed: parts are memory-mapped and walked in
        chunks (ckpt.LOAD_CHUNK_ROWS), so host RAM stays at ~2 chunks per rank
        whatever the model size (reference: the PS loads model_path per node,
        box_wrapper.cc:1201-1242).
        * one rank: every part, chunk by chunk;
        * parts written by a job of this world size (meta "world"): each rank
          reads only its own part -- it holds exactly the keys the rank owns;
        * otherwise each rank reads parts rank, rank + W, ... and routes the
          rows of every chunk to their owners with one bounded all-to-all per
          round (chunk / W rows per rank per round).
        ``merge`` combines the model with the rows already in the table
        (``_merge_rows``, by ``update_type``); otherwise rows are replaced.
        Returns the number of rows this rank loaded."""
        meta = ckpt.read_meta(model_path)
        parts = ckpt.list_parts(model_path)
        if not parts:
            return 0
        t = self._authoritative()
        dev = getattr(t, "device", torch.device("cpu"))
        chunk = max(1, int(ckpt.LOAD_CHUNK_ROWS))
        loaded = 0

        def apply(h: torch.Tensor, v: torch.Tensor) -> int:
            if h.numel() == 0:
                return 0
            h, v = h.to(dev), v.to(dev).float()
            if merge and update_type != "replace":
                found = t.probe(h) >= 0
                cur = t.read(h).to(dev).float()
                v = self._merge_rows(cur, v, found, update_type, int(model_index))
            t.insert_mixed(h, self.cfg.sgd)
            t.assign(h, v)
            if self.mode == "tiered":
                self._push_live(h, v)
            return int(h.numel())

        def mixed(keys: np.ndarray) -> torch.Tensor:
            return ref.mix64(torch.from_numpy(keys.view("int64").copy()))

        if self.world == 1 or int(meta.get("world", -1)) == self.world:
            mine = parts if self.world == 1 else [p for p in parts if p == self.rank]
            for p in mine:
                for k, v in ckpt.iter_part_chunks(model_path, p, chunk):
                    loaded += apply(mixed(k), torch.from_numpy(v))
            return loaded
        # route rows to owners: rounds of chunk / W rows per rank
        W, me = self.world, self.rank
        per = max(1, chunk // W)
        my_parts = parts[me::W]
        gdev = self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        n_rounds = sum((ckpt.part_rows(model_path, p) + per - 1) // per for p in my_parts)
        nr = torch.tensor([n_rounds], dtype=torch.int64, device=gdev)
        dist.all_reduce(nr, op=dist.ReduceOp.MAX, group=self.group)
        stride = int(meta.get("stride") or np.load(os.path.join(model_path, f"part-{parts[0]:05d}.vals.npy"),
                                                   mmap_mode="r", allow_pickle=False).shape[1])
        src = (c for p in my_parts for c in ckpt.iter_part_chunks(model_path, p, per))
        for _ in range(int(nr.item())):
            k, v = next(src, (np.zeros(0, np.uint64), np.zeros((0, stride), np.float32)))
            h, vt = mixed(k), torch.from_numpy(v).reshape(-1, stride)
            owner = ref.owner_of(h, W)
            order = torch.argsort(owner, stable=True)
            h, vt = h[order], vt[order]
            counts = torch.bincount(owner, minlength=W)
            rcd = torch.empty(W, dtype=torch.int64, device=gdev)
            dist.all_to_all_single(rcd, counts.to(gdev), group=self.group)
            sc, rcl = counts.tolist(), rcd.cpu().tolist()
            hk = torch.empty(int(sum(rcl)), dtype=torch.int64, device=gdev)
            dist.all_to_all_single(hk, h.to(gdev), rcl, sc, group=self.group)
            rv = torch.empty(int(sum(rcl)), stride, dtype=torch.float32, device=gdev)
            dist.all_to_all_single(rv, vt.to(gdev), rcl, sc, group=self.group)
            loaded += apply(hk, rv)
        return loaded

    def _merge_rows(self, cur: torch.Tensor, inc: torch.Tensor, found: torch.Tensor, update_type: str,
                    model_index: int) -> torch.Tensor:
        """MergeModel / MergeMultiModels row rule (the closed BoxPS merge is
        not visible; this is this engine's documented contract -- parity
        unpinned):

        * ``add`` (MergeModel): show / click / delta_score summed; a key the
          table already holds keeps its weights and optimizer state, a new
          key takes the incoming row;
        * ``average``: show / click / delta_score summed; weights and g2sums
          become the running mean over the merged models, ``model_index``
          being how many models were merged before this one;
        * ``max_show``: per key, the row with the larger show wins;
        * ``replace``: the incoming row wins (plain load)."""
        l = row_layout(self.cfg.embedx_dim)
        w = min(cur.shape[1], inc.shape[1])
        out = inc.clone()
        f = found
        if not bool(f.any()):
            return out
        c, i = cur[f][:, :w], inc[f][:, :w]
        stats = [l["show"], l["click"], l["delta_score"]]
        if update_type in ("add", "merge", "sum", "0"):
            m = c.clone()
            m[:, stats] = c[:, stats] + i[:, stats]
        elif update_type in ("average", "avg", "1"):
            n = float(max(0, model_index))
            m = (c * n + i) / (n + 1.0)
            m[:, stats] = c[:, stats] + i[:, stats]
            m[:, l["slot"]] = c[:, l["slot"]]
            m[:, l["unseen_days"]] = c[:, l["unseen_days"]]
            m[:, l["mf_size"]] = torch.maximum(c[:, l["mf_size"]], i[:, l["mf_size"]])
        elif update_type in ("max_show", "max", "2"):
            m = torch.where((i[:, l["show"]] > c[:, l["show"]]).unsqueeze(1), i, c)
        else:
            raise ValueError(f"merge: unknown update_type {update_type!r} (add / average / max_show / replace)")
        rows = out[f]
        rows[:, :w] = m
        out[f] = rows
        return out

    def merge_model(self, path: str):
        """MergeModel(path): add-merge a batch model into the table."""
        return self.load_model(path, merge=True, update_type="add")

    def merge_multi_models(self, path, update_type: str = "add", model_index: int = 0):
        """MergeMultiModels(path, update_type, model_index): merge one model of
        a multi-model set (``model_index`` = models merged before it); a list
        of paths merges them in order with increasing index."""
        if isinstance(path, (list, tuple)):
            return sum(self.load_model(p, merge=True, update_type=str(update_type), model_index=model_index + j)
                       for j, p in enumerate(path))
        return self.load_model(path, merge=True, update_type=str(update_type), model_index=int(model_index))

    # rows per load_ssd2mem chunk: one chunk's keys + values are in host RAM at a time
    SSD2MEM_CHUNK_ROWS = 1 << 20

    def load_ssd2mem(self, date: Optional[str] = None, max_rows: Optional[int] = None) -> int:
        """LoadSSD2Mem (box_wrapper.cc:1320-1324): move SSD rows into the host
        tier, streamed in chunks of ``SSD2MEM_CHUNK_ROWS`` and bounded by the
        host-tier row cap (``cfg.tier.ssd_spill_threshold``; ``max_rows`` caps
        it further): rows that would not fit stay on SSD, so the next
        write-back does not spill them straight back.  Returns the rows moved."""
        if self.ssd is None or self.host is None:
            return 0
        self._sync_tiers()
        cap = int(self.cfg.tier.ssd_spill_threshold)
        room = max(0, cap - self.host.size()) if cap > 0 else len(self.ssd)
        if max_rows is not None:
            room = min(room, int(max_rows))
        if room == 0 or len(self.ssd) == 0:
            return 0
        lock = self.tier._tier_lock if self.tier is not None else contextlib.nullcontext()
        moved = 0
        with lock:
            h_all = self.ssd.keys()
            step = max(1, int(self.SSD2MEM_CHUNK_ROWS))
            for a in range(0, min(int(h_all.numel()), room), step):
                h = h_all[a:min(a + step, room)]
                found, vals = self.ssd.get(h)
                hk = h[found]
                if hk.numel() == 0:
                    continue
                rows, _ = self.host._native.insert(hk)
                self.host._native.scatter(rows, vals[found])
                if self.tier is not None:
                    self.host._native.stamp(rows, self.tier.epoch)
                self.ssd.delete(hk)
                moved += int(hk.numel())
        return moved

    def shrink_table(self) -> int:
        """ShrinkTable (box_wrapper.h:638): decay show/click, age, delete
        (ctr_accessor.cc:63-80) over the whole table -- in tiered mode the
        host tier and every SSD record.  Inside a pass the live GPU rows are
        shrunk by the same rule, so the next write-back keeps the result (and
        between passes with the GPU tier, whose activation carries live rows
        into the next pass)."""
        t = self._authoritative()
        gone = t.shrink(self.cfg.shrink)
        if self.mode == "tiered" and self.engine is not None and (self.in_pass or self.tier is not None):
            self.engine.table.shrink(self.cfg.shrink)
        if self.tier is not None and not self.in_pass:
            self.tier.restage()  # a staged next pass read its host rows before the shrink
        return gone

    def shrink_resource(self):
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def check_need_limit_mem(self) -> bool:
        if self.device.type != "cuda":
            return False
        free, total = torch.cuda.mem_get_info(self.device)
        return free < 0.05 * total

    def release_pool(self):
        self.shrink_resource()

    def finalize(self):
        self.engine = None
        BoxWrapper._instance = None

    # ---------------------------------------------------------------- metrics / phases
    def init_metric(self, *a, **k):
        return self.metrics.init_metric(*a, **k)

    def get_metric_msg(self, name):
        return self.metrics.get_metric_msg(name)

    def get_continue_metric_msg(self, name):
        return self.metrics.get_continue_metric_msg(name)

    def get_nan_inf_metric_msg(self, name):
        return self.metrics.get_nan_inf_metric_msg(name)

    def get_metric_name_list(self, metric_phase: int = -1):
        return self.metrics.get_metric_name_list(metric_phase)

    def flip_phase(self):
        self.metrics.flip_phase()

    def set_phase(self, p):
        self.metrics.set_phase(p)

    @property
    def phase(self):
        return self.metrics.phase

    # ---------------------------------------------------------------- misc API parity
    def set_dataset_name(self, name: str):
        self.dataset_name = name

    def set_input_table_dim(self, dim: int):
        self.input_table_dim = dim
        self.input_table.set_dim(dim)

    # ---------------------------------------------------------------- auxiliary tables
    @property
    def replica_cache(self):
        """GpuReplicaCache for pull_cache_value (created on first use)."""
        if self._replica is None:
            from .extras import GpuReplicaCache

            self._replica = GpuReplicaCache(self.cfg.embedx_dim + 3, self.device)
        return self._replica

    @property
    def input_table(self):
        if self._input_table is None:
            from .extras import InputTable

            self._input_table = InputTable(self.input_table_dim)
        return self._input_table

    def pull_extended(self, keys, lod, B, S, emb_size: int, ext_size: int, mask=None):
        """pull_box_extended_sparse: (records [L, emb_size], expand [L, ext_size])."""
        eng = self._require_engine()
        if getattr(eng, "codec", None) is not None and eng.codec.kind == 3:
            # variable feature type: per-feature size, one output per slot
            from .extras import pull_extended_var

            return pull_extended_var(eng, keys, lod, B, S, emb_size, ext_size, mask)
        if getattr(eng, "codec", None) is not None and eng.codec.De >= ext_size:
            # GPU PS rows carry the expand block: one pull / push for both
            from .extras import pull_extended_codec

            return pull_extended_codec(eng, keys, lod, B, S, emb_size, ext_size)
        if self._expand is None:
            from .extras import ExpandEmbedding

            dim = self.cfg.expand_embed_dim or ext_size
            self._expand = ExpandEmbedding(self._require_engine(), dim)
        return self._expand.pull(keys, lod, B, S, emb_size, ext_size)

    def init_afs_api(self, fs_name: str = "", fs_user: str = "", pass_wd: str = "", conf_path: str = "",
                     hadoop_bin: str = ""):
        """Configure the process-wide file client (reference InitAfsAPI,
        box_wrapper.h:721-734: fs_ugi = "user,passwd"): model save/load paths
        and the pass loaders' hdfs:// / afs:// files then go through it."""
        from ..utils.fs import BoxFileMgr

        self.fs = BoxFileMgr()
        ugi = f"{fs_user},{pass_wd}" if (fs_user or pass_wd) else ""
        if not self.fs.init(fs_name, ugi, conf_path, hadoop_bin=hadoop_bin):
            raise RuntimeError("Called AFSAPI Init Interface Failed.")
        self.use_afs_api = True
        return 0

    def print_device_info(self) -> str:
        s = f"rank={self.rank}/{self.world} device={self.device} mode={self.mode}"
        if self.engine is not None:
            s += f" table={self.engine.table.size()} rows, {self.engine.table.memory_bytes() / 2**30:.2f} GiB"
        if self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            s += f" hbm_free={free / 2**30:.1f}/{total / 2**30:.1f} GiB"
        logger().info(s)
        return s

    def print_sync_timer(self) -> str:
        s = self.timers.format()
        logger().info(f"[rank {self.rank}] {s}")
        return s

    # ---------------------------------------------------------------- helpers
    def _require_engine(self) -> SparseEngine:
        if self.engine is None:
            self.initialize_gpu_and_load_model()
        return self.engine
