"""Pass datasets: PadBoxSlotDataset / BoxPSDataset / InputTableDataset.

Python face of the native ``SlotDataset`` (csrc/host/slot_dataset.cc).
Reference API: ``py/fluid/dataset.py:38-270,1231-1500`` (setters, the
``DatasetFactory``), ``fw/data_set.cc:1905-2860`` (PadBoxSlotDataset
behaviour: rank-strided filelist, load/preload, feed-pass key registration,
shuffle, PrepareTrain batching with equal batch counts across ranks, disk
archive mode, release).

Batches come out in the engine layout: all sparse slots as one flat
slot-major key array + LoD offsets (one H2D copy each), dense slots as one
[B, width] float matrix.
"""
from __future__ import annotations

import math
import os
import queue
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import _native
from ..utils import flags as _flags
from ..utils.dayid import make_day_id_str


@dataclass
class SlotVar:
    """A data variable declared with fluid.layers.data (name, dtype, shape, lod)."""

    name: str
    dtype: str = "int64"
    shape: Sequence[int] = (1,)
    lod_level: int = 1

    @property
    def is_sparse(self) -> bool:
        return self.dtype in ("int64", "uint64") and self.lod_level > 0

    @property
    def dense_dim(self) -> int:
        d = 1
        for s in self.shape:
            if s > 0:
                d *= s
        return d


@dataclass
class SlotBatch:
    keys: torch.Tensor
    lod: torch.Tensor
    dense: torch.Tensor
    B: int
    S: int
    sparse_names: List[str]
    dense_names: List[str]
    dense_dims: List[int]
    extra: Dict[str, torch.Tensor] = field(default_factory=dict)
    lod_host: Optional[torch.Tensor] = None  # CPU copy of lod (slot boundaries without a device sync)
    # (native dataset, begin, count, extend_dim) of the records the batch was
    # built from: store_q_value writes PCOC q values back into them
    src: Optional[tuple] = None

    def dense_var(self, name: str) -> torch.Tensor:
        col = 0
        for n, d in zip(self.dense_names, self.dense_dims):
            if n == name:
                return self.dense[:, col:col + d]
            col += d
        raise KeyError(name)

    def to(self, device, non_blocking=False) -> "SlotBatch":
        mv = lambda t: t.to(device, non_blocking=non_blocking) if isinstance(t, torch.Tensor) else t  # noqa: E731
        lh = self.lod if self.lod.device.type == "cpu" else self.lod_host
        return SlotBatch(mv(self.keys), mv(self.lod), mv(self.dense), self.B, self.S, self.sparse_names,
                         self.dense_names, self.dense_dims, {k: mv(v) for k, v in self.extra.items()}, lh,
                         self.src)

    # compat with the synthetic Batch used by the models
    @property
    def label(self) -> torch.Tensor:
        return self.extra["label"]

    @property
    def cvm(self) -> torch.Tensor:
        return self.extra["cvm"]


class DatasetBase:
    """Common setters (py/fluid/dataset.py:81-270)."""

    def __init__(self):
        self.use_vars: List[SlotVar] = []
        self.batch_size = 1
        self.thread_num = 1
        self.filelist: List[str] = []
        self.pipe_command = "cat"
        self.so_parser_name = ""
        self.rank_offset = ""
        self.ads_offset = ""
        self.pv_batch_size = 0
        self.sample_rate = 1.0
        self.parse_ins_id = False
        self.parse_logkey = False
        self.merge_by_lineid = False
        self.date = None
        self.label_name: Optional[str] = None
        self.enable_pv_merge = False
        self.current_phase = 1
        self.fea_eval = False

    def set_use_var(self, var_list):
        self.use_vars = []
        for v in var_list:
            if isinstance(v, SlotVar):
                self.use_vars.append(v)
            else:  # fluid Variable
                self.use_vars.append(SlotVar(v.name, v.dtype, tuple(v.shape), getattr(v, "lod_level", 0)))

    def set_batch_size(self, b):
        self.batch_size = int(b)

    def set_thread(self, n):
        self.thread_num = int(n)

    def set_filelist(self, files):
        self.filelist = list(files)

    def set_pipe_command(self, cmd):
        self.pipe_command = cmd

    def set_so_parser_name(self, name):
        self.so_parser_name = name

    def set_rank_offset(self, name):
        self.rank_offset = name

    def set_ads_offset(self, name):
        self.ads_offset = name

    def set_pv_batch_size(self, n):
        self.pv_batch_size = int(n)

    def set_sample_rate(self, r):
        self.sample_rate = float(r)

    def set_parse_ins_id(self, v):
        self.parse_ins_id = bool(v)

    def set_parse_logkey(self, v):
        self.parse_logkey = bool(v)

    def set_merge_by_lineid(self, v=True):
        self.merge_by_lineid = bool(v)

    def set_enable_pv_merge(self, v):
        self.enable_pv_merge = bool(v)

    def set_current_phase(self, p):
        self.current_phase = int(p)

    def set_fea_eval(self, record_candidate_size=0, fea_eval=True):
        self.record_candidate_size = int(record_candidate_size)
        self.fea_eval = fea_eval

    def set_date(self, date: str):
        self.date = str(date)

    def set_label_var(self, name: str):
        self.label_name = name


class PadBoxSlotDataset(DatasetBase):
    """In-memory pass dataset bound to the BoxPS engine."""

    def __init__(self, rank: Optional[int] = None, world: Optional[int] = None, group=None):
        super().__init__()
        self._native = _native.host().SlotDataset()
        self.group = group
        ready = dist.is_available() and dist.is_initialized()
        self.rank = rank if rank is not None else (dist.get_rank(group) if ready else 0)
        self.world = world if world is not None else (dist.get_world_size(group) if ready else 1)
        self.disable_shuffle_flag = False
        self.disable_polling_flag = False
        self.archive_mode = False
        self.box = None  # BoxWrapper
        self._configured = False
        self._seed = 0

    # -- configuration ----------------------------------------------------
    def _configure(self):
        h = _native.host()
        descs = []
        for v in self.use_vars:
            if v.is_sparse:
                descs.append(h.SlotDesc(v.name, "uint64", True, False, 1))
            else:
                t = "uint64" if v.dtype in ("int64", "uint64") else "float"
                descs.append(h.SlotDesc(v.name, t, True, True, v.dense_dim))
        self._native.set_slots(descs)
        pc = h.ParseConfig()
        pc.parse_ins_id = self.parse_ins_id
        pc.parse_logkey = self.parse_logkey
        pc.sample_rate = self.sample_rate
        self._native.set_parse(pc)
        if self.so_parser_name:  # user instance-parser plugin (csrc/host/parser_plugin.h)
            self._native.set_so_parser(os.path.abspath(self.so_parser_name))
        self._native.set_pipe_command(self.pipe_command)
        self._native.set_thread_num(self.thread_num)
        self._configured = True

    def _my_files(self) -> List[str]:
        """Rank-strided filelist (data_set.cc:1963-1975)."""
        if self.disable_polling_flag or self.world == 1 or _flags.get_bool("padbox_dataset_disable_polling"):
            return list(self.filelist)
        return [f for i, f in enumerate(self.filelist) if i % self.world == self.rank]

    def disable_shuffle(self):
        self.disable_shuffle_flag = True

    def disable_polling(self):
        self.disable_polling_flag = True

    def set_archivefile(self, v: bool):
        self.archive_mode = bool(v)

    # -- loading (feed pass) ----------------------------------------------
    def load_into_memory(self, register_keys: bool = True):
        """Blocking load + feed-pass key registration with BoxPS
        (BoxHelper::ReadData2Memory, box_wrapper.h:1086-1126)."""
        if not self._configured:
            self._configure()
        files = self._my_files()
        agent = self._open_feed_pass() if register_keys else None
        try:
            if self.archive_mode:
                for f in files:
                    self._native.load_archive(f, True)
            else:
                self._native.set_filelist(files)
                self._native.load_into_memory()
            self._maybe_unroll()
        finally:
            self._native.set_key_agent(None)
        if agent is not None:
            self._close_feed_pass(agent)

    def _maybe_unroll(self):
        """FLAGS_padbox_dataset_enable_unrollinstance: the parser plugin's
        UnrollInstance hook rewrites the loaded pass (data_set.cc:2275-2277);
        runs while the feed-pass agent is attached so new feasigns register."""
        if _flags.get_bool("padbox_dataset_enable_unrollinstance") and self._native.has_so_parser():
            if self._native.unroll_instances() < 0:
                raise RuntimeError("parser plugin UnrollInstance failed")

    def _open_feed_pass(self):
        """BeginFeedPass: the loader threads register every parsed record's
        feasigns into the pass agent (data_set.cc:2293-2349)."""
        if self.box is None:
            return None
        agent = self.box.begin_feed_pass(self.date)
        if agent.native is not None:
            self._native.set_key_agent(agent.native)
        else:  # no native agent: walk the store after the load
            agent._collect_from = self
        self._attach_side_tables(agent)
        return agent

    def _attach_side_tables(self, agent):
        """Replica-cache / input-index data feeds (data_feed.cc:4155-4635):
        with FLAGS_use_gpu_replica_cache the pass gets a fresh native replica
        store the parser plugin appends cache rows to; an input table the box
        holds is queried for string-key offsets."""
        h = _native.host()
        if _flags.get_bool("use_gpu_replica_cache"):
            agent.replica = h.ReplicaStore(int(_flags.get("gpu_replica_cache_dim")))
            self._native.set_replica_cache(agent.replica)
        tab = getattr(self.box, "_input_table", None)
        if tab is not None and getattr(tab, "native", None) is not None:
            self._native.set_input_index(tab.native)

    def _close_feed_pass(self, agent):
        self._native.set_replica_cache(None)
        self._native.set_input_index(None)
        if getattr(agent, "replica", None) is not None:
            self.box.replica_cache.load_native(agent.replica)
        if getattr(agent, "_collect_from", None) is self:
            agent.add_keys(self.collect_keys())
        if getattr(self.box, "auc_runner", None) is not None:
            agent.add_keys(self.box.auc_runner.prepare(self))
        self.box.end_feed_pass(agent)

    def read_ins_into_memory(self):
        self.load_into_memory()

    def preload_into_memory(self):
        if not self._configured:
            self._configure()
        self._native.set_filelist(self._my_files())
        self._preload_agent = self._open_feed_pass()
        self._native.preload_into_memory()

    def wait_preload_done(self, register_keys: bool = True):
        try:
            self._native.wait_preload_done()
            self._maybe_unroll()
        finally:
            self._native.set_key_agent(None)
        agent, self._preload_agent = getattr(self, "_preload_agent", None), None
        if agent is not None and register_keys:
            self._close_feed_pass(agent)

    def add_lines(self, lines: List[str]) -> int:
        """Parse in-memory text lines (tests / pipe-less sources)."""
        if not self._configured:
            self._configure()
        return self._native.add_lines(list(lines))

    def preload_into_disk(self, path: str, num_files: int = 1):
        """Dump the loaded records into a binary archive (disk mode,
        data_set.cc:2092-2217)."""
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        self._native.save_archive(path)

    def load_into_disk(self, path: str):
        self.preload_into_disk(path)

    def release_memory(self):
        self._native.release_memory()

    def get_memory_data_size(self) -> int:
        return int(self._native.size())

    def collect_keys(self) -> torch.Tensor:
        return self._native.collect_keys(True)

    # -- pass lifecycle -----------------------------------------------------
    def begin_pass(self):
        if self.box is not None:
            self.box.begin_pass()

    def end_pass(self, need_save_delta: bool = False):
        if self.box is not None:
            self.box.end_pass(need_save_delta)

    # -- shuffle ------------------------------------------------------------
    def local_shuffle(self, seed: Optional[int] = None):
        self._seed += 1
        self._native.shuffle(seed if seed is not None else (self._seed * 7919 + self.rank))

    def global_shuffle(self, seed: int = 0, by_search_id: Optional[bool] = None, chunk: int = 4096):
        """Inter-rank record shuffle (PaddleShuffler flow,
        data_set.cc:2422-2604): every record goes to rank hash % world --
        hash = xxh64 of the 32-byte line id with merge_by_lineid, mix64(search_id)
        with pv merge or FLAGS_enable_shuffle_by_searchid, random otherwise --
        streamed natively in messages of ``chunk`` records over the shuffle
        message service (data/shuffler.py) while the receivers append them.
        FLAGS_padbox_dataset_disable_shuffle keeps records on their rank."""
        if by_search_id is None:
            by_search_id = _flags.get_bool("enable_shuffle_by_searchid") or bool(self.enable_pv_merge)
        if self.world == 1 or _flags.get_bool("padbox_dataset_disable_shuffle"):
            self.local_shuffle(seed)
            return 0
        from .shuffler import get_shuffler

        svc = get_shuffler(self.rank, self.world)
        mode = 2 if self.merge_by_lineid else (1 if by_search_id else 0)
        threads = max(1, _flags.get_int("padbox_dataset_shuffle_thread_num"))
        got = self._native.global_shuffle(svc.svc, mode, int(seed), int(chunk), threads)
        self.local_shuffle(seed)
        return got

    # -- batching -----------------------------------------------------------
    def prepare_train(self, shuffle: Optional[bool] = None) -> List[tuple]:
        """Split this rank's records into batches such that every rank runs
        the same number of batches (data_set.cc:2692-2823)."""
        if shuffle is None:
            # FLAGS_padbox_disable_ins_shuffle: no per-pass instance shuffle (data_set.cc:42)
            shuffle = not self.disable_shuffle_flag and not _flags.get_bool("padbox_disable_ins_shuffle")
        if shuffle:
            self.local_shuffle()
        n = int(self._native.size())
        bs = self.batch_size
        nb = int(math.ceil(n / bs)) if n else 0
        if self.world > 1 and dist.is_initialized():
            t = torch.tensor([nb], dtype=torch.int64)
            backend = dist.get_backend(self.group)
            if backend == "nccl":
                t = t.cuda()
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            nb = int(t.item())
        if nb == 0:
            return []
        # even split of n records into nb batches (tail spread)
        out = []
        start = 0
        for i in range(nb):
            cnt = n // nb + (1 if i < n % nb else 0)
            out.append((start, max(cnt, 0)))
            start += cnt
        return out

    def build_batch(self, begin: int, count: int, pin: bool = False) -> SlotBatch:
        keys, lod, dense = self._native.build_batch(begin, count, pin)
        names = self._native.sparse_slot_names()
        dnames = self._native.dense_slot_names()
        ddims = self._native.dense_slot_dims()
        b = SlotBatch(keys, lod, dense, count, len(names), names, dnames, ddims)
        if self.label_name and self.label_name in dnames:
            lab = b.dense_var(self.label_name)[:, 0].contiguous()
            b.extra["label"] = lab
            b.extra["cvm"] = torch.stack([torch.ones_like(lab), lab], 1)
        if self.rank_offset:
            b.extra[self.rank_offset] = self._native.build_rank_offset(begin, count, 3)
        if self.parse_ins_id:
            b.extra["ins_ids"] = self._native.batch_ins_ids(begin, count)
        if self.parse_logkey:
            b.extra["cmatch_rank"] = self._native.batch_cmatch_rank(begin, count)
        ext = _flags.get_int("padbox_slotrecord_extend_dim")
        if ext > 0 and count > 0:
            # pack_qvalue: the records' q values ride with the batch
            b.extra["q_values"] = self._native.batch_ext(begin, count, ext)
            b.src = (self._native, begin, count, ext)
        return b

    def batches(self, device=None, prefetch: int = 2, shuffle: Optional[bool] = None):
        """Iterate device batches; a background thread assembles pinned host
        batches (GIL released in C++) and H2D copies run on a side stream."""
        plan = self.prepare_train(shuffle)
        dev = torch.device(device) if device is not None else torch.device("cpu")
        pin = dev.type == "cuda"
        q: "queue.Queue" = queue.Queue(maxsize=max(1, prefetch))

        def worker():
            for (b0, cnt) in plan:
                q.put(self.build_batch(b0, cnt, pin))
            q.put(None)

        th = threading.Thread(target=worker, daemon=True)
        th.start()
        stream = torch.cuda.Stream(dev) if pin else None
        while True:
            hb = q.get()
            if hb is None:
                break
            if pin:
                with torch.cuda.stream(stream):
                    db = hb.to(dev, non_blocking=True)
                cur = torch.cuda.current_stream(dev)
                cur.wait_stream(stream)
                # the device batch is allocated on the copy stream but read on
                # the compute stream: without this its memory returns to the copy
                # stream's pool when the batch is dropped, and a later batch's
                # H2D copy can overwrite it while the step that read it is
                # still queued (the host runs ahead in the eager loop)
                for t in (db.keys, db.lod, db.dense, *db.extra.values()):
                    if isinstance(t, torch.Tensor) and t.is_cuda:
                        t.record_stream(cur)
                yield db
            else:
                yield hb
        th.join()

    def slots_shuffle(self, slots):
        """Replace the feasigns of ``slots`` in every instance by those of a
        random other instance (reservoir-sampled), restoring the slots of the
        previous call first; ``[]`` restores only.  With a BoxWrapper in
        AucRunner mode this is BoxHelper::SlotsShuffle (phase flip, the
        runner's candidates, box_wrapper.h:1185-1209); otherwise
        Dataset::SlotsShuffle with a local reservoir (data_set.cc:1583-1614)."""
        from ..ps.auc_runner import AucRunner

        runner = getattr(self.box, "auc_runner", None) if self.box is not None else None
        if runner is not None:
            self.box.flip_phase()
        else:
            runner = getattr(self, "_slot_shuffler", None)
            if runner is None or not runner.covers(self, slots):
                if runner is not None:
                    runner.shuffle(self, [])
                size = getattr(self, "record_candidate_size", 0) or 10000
                runner = AucRunner([list(slots)], 4, size)
                runner.prepare(self)
                self._slot_shuffler = runner
        return runner.shuffle(self, list(slots))

    def __len__(self):
        return int(self._native.size())


class BoxPSDataset(PadBoxSlotDataset):
    """Legacy BoxPSDataset (PaddleBoxDataFeed over MultiSlot records):
    join phase builds page-view batches with rank_offset, update phase
    instance batches (data_feed.cc:1780-1990)."""

    def prepare_train(self, shuffle=None):
        if self.enable_pv_merge and self.current_phase == 1:
            off = self._native.merge_by_search_id().tolist()
            pvs = [(off[i], off[i + 1] - off[i]) for i in range(len(off) - 1)]
            pvb = max(1, self.pv_batch_size or self.batch_size)
            out = []
            for i in range(0, len(pvs), pvb):
                grp = pvs[i:i + pvb]
                out.append((grp[0][0], sum(c for _, c in grp)))
            return out
        return super().prepare_train(shuffle)


class InputTableDataset(PadBoxSlotDataset):
    """Dataset with a string-key -> dense-vector index table (lookup_input op,
    data_set.cc:2830-2858)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.index_files: List[str] = []

    def set_index_parser_files(self, files):
        self.index_files = list(files)

    def load_index_into_memory(self, table=None):
        """InputTableDataFeed: index files into the box's input table (the
        parser plugin's parse_index when it has one, else "key v1..vD")."""
        if not self._configured:
            self._configure()
        table = table if table is not None else self.box.input_table
        if getattr(table, "native", None) is not None:
            n = int(self._native.load_index_files(list(self.index_files), table.native))
            table.dim = int(table.native.dim())
            return n
        return sum(table.load_text(f) for f in self.index_files)


class DatasetFactory:
    """fluid.DatasetFactory().create_dataset(name)."""

    _classes = {
        "PadBoxSlotDataset": PadBoxSlotDataset,
        "BoxPSDataset": BoxPSDataset,
        "InputTableDataset": InputTableDataset,
    }

    def create_dataset(self, datafeed_class: str = "PadBoxSlotDataset", **kw):
        if datafeed_class not in self._classes:
            raise ValueError(f"datafeed class {datafeed_class} does not exist")
        return self._classes[datafeed_class](**kw)

