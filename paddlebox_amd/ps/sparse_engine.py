"""Per-batch sparse pipeline: dedup -> (key exchange) -> probe -> pull ->
fused seqpool+CVM, and the mirror push path with fused sparse Adagrad.

This is the engine behind ``pull_box_sparse``/``push_box_sparse`` and
``fused_seqpool_cvm`` (reference pipeline: ``box_wrapper_impl.h:25-234``
pull, ``:373-522`` push; BoxPS ``PullSparseGPU/PushSparseGPU`` closed).

MI355X design points
--------------------
* No host synchronisation per batch: unique counts live on the device and
  every kernel is launched for the static upper bound, so a whole training
  step is captured in one HIP graph.
* One shard (world = 1, the default): the dedup runs THROUGH the table -- the
  pass-resident table row is the unique id.  ``k_table_rank`` probes every
  occurrence (LDS-staged bucket, wave ballot) and ranks first occurrences,
  ``k_table_seg`` / ``k_table_scatter`` build the per-unique occurrence
  segments; the fused seqpool+CVM reads each occurrence's row directly.  The
  push is one wave-segmented merge with the Adagrad update in registers
  (``k_push_merge_apply``) plus ``k_push_finish`` for runs that straddle waves.
  ``dedup=False`` (FLAGS_enable_pullpush_dedup_keys) probes per occurrence and
  merges the push by leader election per table row instead.
* Sharded (world > 1): the sender dedups with the sort-free hash dedup
  (``dedup.hip``: insert, rank, segment, scatter) and packs its unique keys
  per owner (``owner = floor(h * N / 2^64)``, ``h = mix64(key)``).  The
  exchange runs on the in-house IPC mesh (``parallel/ipc.py``: one kernel per
  exchange, only ``counts[p]`` records of each peer slot travel, worst-case or
  pre-scanned exact slots, so nothing is dropped) or, as the fallback, on RCCL
  ``all_to_all_single`` with fixed per-peer slots (heuristic slot size, sticky
  device overflow flag checked at pass end).  The owner probes and gathers in
  one launch, answers, and applies the pushed gradients with a leader-elected
  per-row Adagrad (no owner-side dedup).
* Feature-type codecs (int16 embedx, expand block, variable, SparseAdam) run
  through the codec kernels of ``feature_ops.hip`` on the hash-dedup path.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native
from ..parallel.comm import Comm, TorchDistComm, default_comm
from ..ops import reference as ref
from .config import PSConfig, SparseSGDConfig, padded, pull_width, push_width
from .cpu_table import CpuSparseTable
from .feature_types import FeatureCodec
from .gpu_table import GpuSparseTable
from ..runtime.streams import side_stream

# sharded pull over the IPC mesh, PBX_PACK_EXCHANGE=1: the owner pack inside
# the key exchange's put phase (ipc.hip k_ipc_pack_exchange) and the owner's
# probe + gather inside the answer exchange (k_ipc_answer_exchange).  Off by
# default: measured slower than pack -> exchange -> probe + gather -> exchange
# (1-rank rehearsal 0.390-0.391 vs 0.380-0.381 ms/step,
# profiles/r6_sharded_rehearsal.txt) -- the fused puts scatter 8-B keys and
# 48-B records into the uncached inbox one transaction each, where the plain
# exchange streams a packed buffer in full 16-B lanes, and the fused kernels
# run on the exchange's co-resident grid instead of a grid per key
def _pack_exchange() -> bool:
    return os.environ.get("PBX_PACK_EXCHANGE", "0") == "1"


def _early_key_exchange() -> bool:
    """Sharded split prefetch, PBX_EARLY_KEY_EXCHANGE=1: the next batch's owner
    pack + key exchange right after its dedup (at step start on the dW stream)
    instead of with the pooling after the push.  Off by default: it takes 18
    us off the sparse chain, but the step does not gain (1-rank rehearsal
    0.3821 vs 0.3794-0.3811 ms/step) -- the dense all-reduce behind the dW
    GEMM becomes the critical path and the longer step-start chain delays the
    tower forward (profiles/r6_sharded_rehearsal.txt)."""
    return os.environ.get("PBX_EARLY_KEY_EXCHANGE", "0") == "1"


@dataclass
class SeqpoolParams:
    use_cvm: bool = True
    cvm_offset: int = 2
    clk_filter: bool = False
    pad_value: float = 0.0
    need_filter: bool = False
    show_coeff: float = 0.2
    clk_coeff: float = 1.0
    threshold: float = 0.96
    quant_ratio: int = 0
    embed_threshold_filter: bool = False
    embed_threshold: float = 0.0
    embed_thres_size: int = 0

    def out_width(self, E: int) -> int:
        return ref.seqpool_cvm_out_width(E, self.use_cvm, self.cvm_offset, self.clk_filter,
                                         0 if self.use_cvm else self.embed_thres_size)


class _PullSlot:
    """Per-pull device buffers (the dedup workspace, occurrence map and, when
    sharded, the exchange buffers).  The engine rotates through a ring of these
    so that several pulls can be outstanding before their pushes -- e.g. two
    pull ops in one program -- without the second overwriting what the first
    one's backward needs.  ``gen`` detects a push against a recycled slot."""

    def __init__(self, eng: "SparseEngine"):
        dev = eng.device
        h = eng._hip
        with torch.cuda.device(dev):
            self.ws = h.DedupWorkspace(eng.max_keys, dev.index or 0, True)
            if getattr(eng, "table_dedup", False):
                # allocate (and -1 / zero fill) the table-dedup buffers now: a
                # slot first used inside a graph capture would otherwise record
                # those fills into the graph and replay them every step
                self.ws.table_rows_occ()
        self.occ_slot = torch.empty(eng.max_keys, dtype=torch.int32, device=dev)
        self.occ_ins = torch.empty(eng.max_keys, dtype=torch.int32, device=dev)
        self.rows = None  # persistent probe rows of a prefetched batch
        self.pre_out = None  # persistent pooled output of a prefetched seqpool (prefetch_pull)
        # one persistent pooled output per batch shape: graphs captured for
        # different batch sizes (a pass's 64- and 63-row batches) keep the
        # address they were captured with -- re-allocating on a shape change
        # freed the buffer a graph of the other size still wrote / read
        self.pre_outs = {}
        self.gen = 0
        # no-dedup pull: table row of every key occurrence
        self.rows_occ = None if eng.dedup else torch.empty(eng.max_keys, dtype=torch.int64, device=dev)
        if eng.sharded:
            n = eng.world * eng.C
            with torch.cuda.device(dev):
                self.ws_r = h.DedupWorkspace(n, dev.index or 0, True)
            self.send = torch.empty(n, dtype=torch.int64, device=dev)
            self.recv = torch.empty(n, dtype=torch.int64, device=dev)
            self.send_index = torch.empty(eng.max_keys, dtype=torch.int64, device=dev)
            self.ocnt = torch.zeros(eng.world, dtype=torch.int32, device=dev)
            self.rcnt = torch.zeros(eng.world, dtype=torch.int32, device=dev)  # keys received per peer (IPC)
            self.rows_recv = torch.empty(n, dtype=torch.int64, device=dev)  # table row per received key
            self.resp = torch.empty(n, eng.P, device=dev)
            self.resp_back = torch.empty(n, eng.P, device=dev)
            self.rows_r = None
            self.keys_exchanged = False  # prefetch_dedup ran this slot's pack + key exchange

    def pooled_out(self, shape, device) -> torch.Tensor:
        t = self.pre_outs.get(shape)
        if t is None:
            t = self.pre_outs[shape] = torch.empty(shape, dtype=torch.float32, device=device)
        self.pre_out = t
        return t


@dataclass
class PullState:
    """What the push of the same batch needs (DeviceBoxData equivalent,
    box_wrapper.h:378-435)."""

    B: int
    S: int
    L: int
    lod: torch.Tensor
    uid: torch.Tensor = None
    perm: torch.Tensor = None
    counts: torch.Tensor = None  # device [U, n_valid]
    rows: torch.Tensor = None  # world==1: table rows per unique
    send_index: Optional[torch.Tensor] = None
    rows_r: Optional[torch.Tensor] = None
    slot: Optional[_PullSlot] = None  # GPU: the buffers this pull used
    gen: int = 0
    extra: dict = field(default_factory=dict)


TABLE_DEDUP_MAX_ROWS = (1 << 31) - 1


def _dense_rows(dense: torch.Tensor) -> torch.Tensor:
    """Dense columns for the fused seqpool launch, read in place when they are
    a unit-stride column slice of the batch's dense block (the launch takes
    the row stride), copied otherwise."""
    dense = dense.float()
    if (dense.dim() == 2 and (dense.stride(1) == 1 or dense.shape[1] == 1)
            and (dense.stride(0) >= dense.shape[1] or dense.shape[0] == 1)):
        return dense
    return dense.contiguous()  # an expanded (row stride 0) or column-strided view: copied


def _push_run_scratch(max_keys: int, device) -> torch.Tensor:
    """Runs of a key's occurrences that straddle waves in the fused merge +
    update: int64 arrival counters per unique (one launch, default: the
    piece that completes a run applies it; the first form of it fenced every
    piece and measured 0.49 vs 0.38 ms/step), or with PBX_PUSH_FINISH=1 the
    int32 per-wave run owners of the two-launch form (k_push_finish).  With
    the x3 tower the push sits on the step's critical path: one launch is
    0.2515-0.2518 vs 0.2569-0.2577 ms/step (profiles/r6_x3_sparse_knob_ab.txt)."""
    if os.environ.get("PBX_PUSH_FINISH", "0") == "1":
        return torch.empty((max_keys + 63) // 64 + 1, dtype=torch.int32, device=device)
    return torch.zeros(max_keys, dtype=torch.int64, device=device)


def table_dedup_fits(table_rows: int) -> bool:
    """The single-shard table dedup (table.hip k_table_rank) keys its LDS hash
    and per-row scratch by int32 row; past INT32_MAX rows the engine falls
    back to the sort-free hash dedup (dedup.hip), which carries int64 rows."""
    return int(table_rows) < TABLE_DEDUP_MAX_ROWS


def exchange_capacity_for(key_batches, world: int, comm: Optional[Comm] = None) -> int:
    """Exact per-peer capacity of the key exchange for a known set of batches
    (a pass is loaded before it is trained, as in BoxPS FeedPass): the largest
    number of distinct keys any batch sends to one owner, max-reduced over the
    ranks when ``comm`` is given.  Sizing by distinct keys per owner instead of
    by occurrences shrinks the exchanged buffers ~4x on Criteo-shaped batches
    (U/L ~ 0.32) and makes overflow impossible for these batches."""
    worst = 0
    for k in key_batches:
        k = k.reshape(-1)
        k = k[k != -1]
        if k.numel() == 0:
            continue
        h = torch.unique(ref.mix64(k))
        worst = max(worst, int(torch.bincount(ref.owner_of(h, world), minlength=world).max()))
    if comm is not None:
        t = torch.tensor([worst], dtype=torch.int64, device=getattr(comm, "device", None) or "cpu")
        comm.all_reduce(t, "max")
        worst = int(t.item())
    return worst + 64


class SparseEngine:
    """Sparse embedding engine for one rank (one GPU, or the CPU)."""

    def __init__(
        self,
        cfg: PSConfig,
        max_keys: int,
        device: torch.device,
        capacity: int = 1 << 20,
        slot_ids: Optional[List[float]] = None,
        group=None,
        cap_factor: Optional[float] = None,
        auto_insert: bool = False,
        comm: Optional[Comm] = None,
        pull_ring: int = 2,
        exchange_capacity: Optional[int] = None,
        exchange: Optional[str] = None,
        dedup: Optional[bool] = None,
    ):
        """``exchange`` (sharded GPU engines): "ipc" = the in-house xGMI peer-
        write mesh (parallel/ipc.py; default, self-tested at construction with
        a fallback to RCCL), "rccl" = torch.distributed all_to_all_single.
        PBX_SPARSE_EXCHANGE overrides the default.

        ``dedup`` (FLAGS_enable_pullpush_dedup_keys, default true): false =
        the single-shard GPU step probes every key occurrence and merges the
        push per table row by leader election (probe, seqpool, push elect,
        push apply: four launches, no key dedup at all -- the reference's
        no-dedup pull/push, box_wrapper.cu:1049-1060).  Sharded engines,
        feature-type codecs and dims without vector kernels keep the dedup."""
        self.cfg = cfg
        self.dim = cfg.embedx_dim
        self.E = pull_width(self.dim)
        self.P = padded(self.E)  # exchanged pull record stride (16-B rows)
        self.Q = padded(push_width(self.dim))
        self.device = torch.device(device)
        self.max_keys = int(max_keys)
        self.group = group
        self.comm = comm if comm is not None else default_comm(group)
        self.world = self.comm.world if self.comm is not None else 1
        # sharded = the key/value/grad exchange runs (world > 1, or forced for a
        # 1-rank rehearsal of the multi-GPU step, see parallel.comm)
        self.sharded = self.comm is not None
        self.rank = self.comm.rank if self.comm is not None else 0
        self.auto_insert = auto_insert
        self.test_mode = False
        self.is_gpu = self.device.type == "cuda"
        self.xmesh = None  # IPC meshes of the sharded exchange (GPU, see _setup_exchange)
        self.exchange_mode = "rccl" if self.sharded else "none"
        shard_cap = int(math.ceil(capacity / self.world)) if self.world > 1 else capacity
        # non-default feature types (int16 embedx, expand block, SparseAdam):
        # rows go through the codec kernels (ps/feature_types.py)
        if dedup is None:
            from ..utils import flags as _flags

            dedup = _flags.get_bool("enable_pullpush_dedup_keys")
        self.codec = FeatureCodec.from_config(cfg)
        if self.codec is not None and not self.is_gpu_device():
            if self.codec.kind != 0:
                raise NotImplementedError("feature_type / sparse_optimizer='adam' need the GPU parameter server")
            self.codec = None  # CPU: the expand block is served by ps.extras.ExpandEmbedding
        self.xdim = self.codec.DX if self.codec is not None else self.dim
        if self.codec is not None:
            self.codec.device = self.device
            # variable feature type: one more pull column carries the row's size
            self.P = padded((4 if self.codec.kind == 3 else 3) + self.xdim)
            self.Q = padded(4 + self.xdim)
        if self.is_gpu:
            self.table = GpuSparseTable(self.dim, shard_cap, self.device, codec=self.codec)
            self._hip = _native.hip()
            self._guard_dev = str(torch.device("cuda", self.device.index if self.device.index is not None
                                               else torch.cuda.current_device()))
            self._hip.clear_guard_bits(self._guard_dev)  # allocates the seqpool guard word outside any capture
            self._sgd_native = cfg.sgd.to_native(self._hip)
            if self.sharded:
                # per-peer exchange slots: exact when the pass's batches were
                # pre-scanned (exchange_capacity_for); otherwise the worst case
                # (every key of a batch owned by one peer), so the exchange can
                # never overflow -- only counts[p] records of a slot travel over
                # the IPC mesh, so the large slots cost HBM (~1 GB at 8 ranks and
                # 213K keys per batch, nothing on 288 GB) but no bandwidth.
                # cap_factor restores a smaller heuristic slot (sticky overflow flag).
                # The worst-case slot only pays on the IPC mesh; RCCL's
                # all_to_all_single always moves whole slots, so it keeps the
                # heuristic slot (1.25 x the even share, sticky overflow flag).
                xmode = exchange or os.environ.get("PBX_SPARSE_EXCHANGE", "ipc")
                self.C = self._exchange_slot(exchange_capacity, cap_factor, self._ipc_candidate(xmode))
                self._setup_exchange(xmode)
                if self.exchange_mode != "ipc" and exchange_capacity is None and cap_factor is None:
                    self.C = self._exchange_slot(None, None, False)
            # no-dedup single-shard step (see the docstring)
            self.dedup = bool(dedup) or self.sharded or self.codec is not None or self.dim not in (4, 8, 16, 32)
            # single shard: dedup through the table itself (the row is the
            # unique id): probe + rank in one launch, no scratch hash table
            # ... for tables up to INT32_MAX rows (its LDS hash and per-row
            # scratch hold int32 rows); bigger single-GPU tables (~2^31+ slots,
            # ~190+ GB at the default layout) take the hash dedup instead
            self.table_dedup = (not self.sharded and os.environ.get("PBX_TABLE_DEDUP", "1") != "0"
                                and table_dedup_fits(self.table.rows))
            # ... split off the critical path (_pull_split, PBX_SPLIT_PULL=1):
            # measured slower on one MI355X (same-box interleaved A/B, 3 reps:
            # 0.283 vs 0.263-0.268 ms/step, profiles/r3_s2_split_pull_ab.txt) --
            # the side-stream dedup's atomics slow the concurrent head / tower
            # forward more than the overlap saves -- so it stays opt-in
            self.split_pull = os.environ.get("PBX_SPLIT_PULL", "0") == "1"
            # table dedup: the seqpool reads each occurrence's row directly
            self.seqpool_rows_occ = os.environ.get("PBX_SEQPOOL_ROWS_OCC", "1") != "0"
            # ring of per-pull buffers (sort-free hash dedup everywhere: the
            # sender packs its unique keys per owner with a counting pass)
            self._slots = [_PullSlot(self) for _ in range(max(1, int(pull_ring)))]
            self._prepared = {}  # key-buffer address -> (slot, L) of a prefetched batch
            self._prepared_keep = {}  # key-buffer address -> its storage (kept alive while prepared)
            self._prepared_out = {}  # key-buffer address -> pooled output of a prefetch_pull
            self._next_slot = 0
            self._cur = self._slots[0]
            if self.sharded:
                n = self.world * self.C
                self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)
                self.push_send = torch.empty(n, self.Q, device=self.device)
                self.push_recv = torch.empty(n, self.Q, device=self.device)
                self.push_merged = torch.empty(n, self.Q, device=self.device)
                # fused merge straddle scratch (all-zero between steps) + run arrival counters
                self.push_acc = torch.zeros(self.max_keys, self.Q, device=self.device)
                self.push_inc = _push_run_scratch(self.max_keys, self.device)
            else:
                self.push_buf = torch.empty(self.max_keys, self.Q, device=self.device)
                if self.codec is not None:  # decoded pull records of the batch's unique keys
                    self.pull_buf = torch.empty(self.max_keys, self.P, device=self.device)
                # fused merge+Adagrad scratch: straddling-run accumulators and
                # run arrival counters (both kept all-zero between steps)
                self.push_acc = torch.zeros(self.max_keys, self.Q, device=self.device)
                self.push_inc = _push_run_scratch(self.max_keys, self.device)
                if not self.dedup:  # per-occurrence accumulators, kOccRep replicas each (kept all-zero)
                    self.push_acc_occ = torch.zeros(self.max_keys * int(self.table.t.occ_replicas), self.Q,
                                                    device=self.device)
        else:
            self.table = CpuSparseTable(self.dim)
            self.dedup = True
            self.table_dedup = False
        self._pending_dedup = None
        self.slot_ids = torch.tensor(slot_ids if slot_ids is not None else [], dtype=torch.float32,
                                     device=self.device)
        self._seed = 1234

    # ------------------------------------------------------------------ build
    def _ipc_candidate(self, mode: str) -> bool:
        return mode == "ipc" and isinstance(self.comm, TorchDistComm) and self.world <= 8

    def _exchange_slot(self, exact: Optional[int], cap_factor: Optional[float], ipc: bool) -> int:
        """Per-peer exchange slot (records): exact when the pass was
        pre-scanned (exchange_capacity_for); the worst case (every key of a
        batch owned by one peer) on the IPC mesh, where only the valid records
        of a slot travel; otherwise the heuristic ``cap_factor`` share."""
        if exact is not None:
            return (int(exact) + 63) // 64 * 64
        if cap_factor is None and ipc:
            return (self.max_keys + 63) // 64 * 64
        f = 1.25 if cap_factor is None else float(cap_factor)
        return min((self.max_keys + 63) // 64 * 64, int(math.ceil(self.max_keys / self.world * f)) + 64)

    def _setup_exchange(self, mode: str):
        """Sparse key / value / gradient exchange transport.  "ipc": three
        IPC meshes (one per record kind, so each received view is a contiguous
        [world * C] array) moving only the valid records of each peer slot;
        self-tested on every rank, all ranks fall back to RCCL together if any
        rank's test fails (e.g. no peer access between the GPUs)."""
        self.exchange_mode = "rccl"
        if not self._ipc_candidate(mode):
            return
        from ..parallel.ipc import IpcMesh, IpcMeshError

        meshes = []
        try:
            for rec in (8, self.P * 4, self.Q * 4):
                meshes.append(IpcMesh(self.C * rec, group=self.group, device=self.device))
        except IpcMeshError as e:
            for m in meshes:
                m.close()
            print(f"[sparse] IPC exchange unavailable ({e}); using RCCL all_to_all", flush=True)
            return
        # (each mesh passed its constructor's payload self-test on every rank)
        self.xmesh = meshes
        self.exchange_mode = "ipc"
        dev = self.device
        self._rcnt = torch.zeros(self.world, dtype=torch.int32, device=dev)

    def check_exchange(self):
        """Raise if an IPC exchange timed out (outside the hot loop)."""
        for m in self.xmesh or ():
            m.check()

    def is_gpu_device(self) -> bool:
        return self.device.type == "cuda"

    def set_slot_ids(self, slot_ids: List[float]):
        self.slot_ids = torch.tensor(slot_ids, dtype=torch.float32, device=self.device)

    def register_keys(self, keys: torch.Tensor, init_embedx: bool = False):
        """Feed-pass key registration: make every key of the coming pass
        resident at its owner shard (BoxPS FeedPass/EndFeedPass,
        box_wrapper.cc:120-169).  Collective over the group when world > 1."""
        keys = keys.reshape(-1).to(self.device)
        keys = keys[keys != -1]
        if self.is_gpu:
            h = torch.unique(ref.mix64(keys))
        else:
            h = torch.unique(ref.mix64(keys))
        if self.sharded:
            owner = ref.owner_of(h, self.world)
            order = torch.argsort(owner, stable=True)
            h = h[order]
            counts = torch.bincount(owner, minlength=self.world)
            in_counts = torch.empty_like(counts)
            self.comm.all_to_all_single(in_counts, counts)
            recv = torch.empty(int(in_counts.sum()), dtype=torch.int64, device=self.device)
            self.comm.all_to_all_single(recv, h, in_counts.tolist(), counts.tolist())
            h = torch.unique(recv)
        self.table.insert_mixed(h, self.cfg.sgd, init_embedx=init_embedx)

    def insert_local_mixed(self, h: torch.Tensor, init_embedx: bool = False):
        """Insert mixed keys already known to belong to this shard."""
        self.table.insert_mixed(h, self.cfg.sgd, init_embedx=init_embedx)

    # ------------------------------------------------------------------ pull
    def pull_seqpool_cvm(self, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int, out: torch.Tensor,
                         col_offset: int, sp: SeqpoolParams, dense: Optional[torch.Tensor] = None,
                         dense_col: int = 0) -> PullState:
        """Fused pull + seqpool + CVM written into out[:, col_offset:...]
        (+ the dense features into out[:, dense_col:...] by the same launch).

        keys: int64 [Lcap] slot-major flat keys, -1 padded; lod: int64 [S*(B+1)].
        """
        if not self.is_gpu:
            st = self._cpu_pull_seqpool(keys, lod, B, S, out, col_offset, sp)
            if dense is not None:
                out[:, dense_col:dense_col + dense.shape[1]] = dense
            return st
        h = self._hip
        pre_out = self._prepared_out.pop(keys.data_ptr(), None) if self._prepared_out else None
        if pre_out is not None and pre_out is out and col_offset == 0:
            # prefetch_pull already pooled this batch into out: only the pull state
            return self._pull_common(keys, lod, B, S, fill_occ=False)
        if not self.dedup and sp.cvm_offset == 2:
            return self._pull_nodedup(keys, lod, B, S, out, col_offset, sp, dense, dense_col)
        if (self.table_dedup and self.split_pull and self.codec is None
                and keys.data_ptr() not in self._prepared):
            return self._pull_split(keys, lod, B, S, out, col_offset, sp, dense, dense_col)
        # the occurrence map is written by the seqpool launch itself
        st = self._pull_common(keys, lod, B, S, fill_occ=False)
        sl = st.slot
        if not self.sharded and self.codec is not None:
            self.table.t.codec_pull(self.codec.native(), st.rows, None, sl.ws.u_count, st.L, self.pull_buf)
            src, src_index = self.pull_buf, None
        elif not self.sharded:
            src, src_index = self.table.values, st.rows
        else:
            src, src_index = sl.resp_back, sl.send_index
        uid = sl.ws.uid
        if (st.extra.get("rows_occ") is not None and self.seqpool_rows_occ and not self.sharded
                and self.codec is None):
            # table dedup: the occurrence's row is known directly (one dependent
            # load less per occurrence than uid -> rows_u)
            src_index, uid = st.extra["rows_occ"], None
        if dense is not None:
            dense = _dense_rows(dense)
        h.seqpool_cvm_fwd(src, src_index, uid, lod, S, B, self.E, out, col_offset, sp.use_cvm,
                          sp.cvm_offset, sp.clk_filter, sp.pad_value, sp.need_filter, sp.show_coeff, sp.clk_coeff,
                          sp.threshold, sp.quant_ratio, sp.embed_threshold_filter, sp.embed_threshold,
                          sp.embed_thres_size if not sp.use_cvm else 0, dense, dense_col,
                          occ_slot=sl.occ_slot, occ_ins=sl.occ_ins)
        return st

    def _pull_nodedup(self, keys, lod, B, S, out, col_offset, sp, dense, dense_col) -> PullState:
        """No-dedup pull: probe every occurrence, pool straight from the rows."""
        h = self._hip
        L = keys.numel()
        assert L <= self.max_keys, f"batch has {L} keys > engine max_keys {self.max_keys}"
        sl = self._take_slot()
        rows = sl.rows_occ[:L]
        self.table.t.probe_raw(keys, rows)
        if self.auto_insert and not self.test_mode:
            miss = (rows < 0) & (keys != -1)
            if bool(miss.any()):
                self.table.insert_mixed(torch.unique(ref.mix64(keys[miss])), self.cfg.sgd)
                self.table.t.probe_raw(keys, rows)
        if dense is not None:
            dense = _dense_rows(dense)
        h.seqpool_cvm_fwd(self.table.values, rows, None, lod, S, B, self.E, out, col_offset, sp.use_cvm,
                          sp.cvm_offset, sp.clk_filter, sp.pad_value, sp.need_filter, sp.show_coeff, sp.clk_coeff,
                          sp.threshold, sp.quant_ratio, sp.embed_threshold_filter, sp.embed_threshold,
                          sp.embed_thres_size if not sp.use_cvm else 0, dense, dense_col,
                          occ_slot=sl.occ_slot, occ_ins=sl.occ_ins)
        st = PullState(B=B, S=S, L=L, lod=lod, slot=sl, gen=sl.gen)
        st.rows = rows
        st.extra["nodedup"] = True
        return st

    def _pull_split(self, keys, lod, B, S, out, col_offset, sp, dense, dense_col) -> PullState:
        """Single-shard pull with the dedup split off the critical path: one
        launch probes every occurrence and pools straight from its table row
        (the seqpool's fused probe, which also records the rows); the table
        dedup (per-row ranks, run starts, perm) that only the push needs runs
        on a side stream, overlapping the dense forward, and the push joins
        it.  The reference orders DedupKeysAndFillIdx before PullSparseGPU
        (box_wrapper_impl.h:152-155); here the dense step never waits for it."""
        h = self._hip
        keys = keys.reshape(-1)
        L = keys.numel()
        assert L <= self.max_keys, f"batch has {L} keys > engine max_keys {self.max_keys}"
        self._join_dedup()
        sl = self._take_slot()
        ws = sl.ws
        rows = ws.table_rows_occ()[:L]  # all -1 outside the lod between pulls
        # ... unless a probing dedup (prefetched / plain table-dedup pull) used
        # this slot last: its rows_occ still holds rows, and the padding
        # positions would then count as occurrences of stale rows
        ws.clean_rows_occ()
        if dense is not None:
            dense = _dense_rows(dense)

        def pool():
            h.seqpool_cvm_fwd(self.table.values, None, None, lod, S, B, self.E, out, col_offset, sp.use_cvm,
                              sp.cvm_offset, sp.clk_filter, sp.pad_value, sp.need_filter, sp.show_coeff,
                              sp.clk_coeff, sp.threshold, sp.quant_ratio, sp.embed_threshold_filter,
                              sp.embed_threshold, sp.embed_thres_size if not sp.use_cvm else 0, dense, dense_col,
                              occ_slot=sl.occ_slot, occ_ins=sl.occ_ins, probe_keys=keys, probe_table=self.table.t,
                              rows_out=rows)

        pool()
        if self.auto_insert and not self.test_mode:
            miss = (rows < 0) & (keys != -1)
            if bool(miss.any()):
                self.table.insert_mixed(torch.unique(ref.mix64(keys[miss])), self.cfg.sgd)
                pool()
        st = PullState(B=B, S=S, L=L, lod=lod, uid=ws.uid, perm=ws.perm, counts=ws.u_count, slot=sl, gen=sl.gen)
        st.rows = ws.rows_u[:L]
        if self.test_mode:
            rows.fill_(-1)  # no push, no dedup: restore the all -1 invariant here
            return st
        cur = torch.cuda.current_stream(self.device)
        # the tower's dW stream: a process gets GPU_MAX_HW_QUEUES (4) hardware
        # queues, and a fifth stream lands on the batch-copy queue, where the
        # next batch's H2D DMA blocks this dedup (measured 0.35 vs 0.26 ms per
        # step); the dedup finishes long before the dW GEMM is issued there
        side = side_stream(self.device, "tower_dw")
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            ws.run_table(keys, self.table.t, True)
        ev = torch.cuda.Event()
        ev.record(side)
        st.extra["dedup_event"] = ev
        self._pending_dedup = ev
        return st

    def _join_dedup(self, st: Optional[PullState] = None):
        """Make the current stream wait for a split pull's side-stream dedup
        (the push of that batch, or the next pull if the push never ran)."""
        ev = st.extra.pop("dedup_event", None) if st is not None else None
        if ev is None:
            ev = self._pending_dedup
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            if ev is self._pending_dedup:
                self._pending_dedup = None

    def can_prefetch(self) -> bool:
        """Prefetched pulls need a fixed key set during training: GPU, one
        shard, no auto-insert (keys registered at the feed pass)."""
        return (self.is_gpu and not self.sharded and not (self.auto_insert and not self.test_mode)
                and len(self._slots) >= 2 and self.dedup)

    def prefetch(self, keys: torch.Tensor, slot: int):
        """Dedup + probe of a batch ahead of its pull, into pull slot ``slot``
        (pipelined training: issued on a side stream while the previous batch
        trains).  The batch's ``pull_seqpool_cvm`` on the same key buffer then
        starts at the seqpool.  Buffers are persistent, so this is
        graph-capturable."""
        if not self.can_prefetch():
            raise RuntimeError("prefetch needs a GPU, unsharded engine without auto-insert")
        L = keys.numel()
        assert L <= self.max_keys
        sl = self._slots[slot % len(self._slots)]
        if sl.rows is None:
            sl.rows = torch.empty(self.max_keys, dtype=torch.int64, device=self.device)
        if self.table_dedup:
            sl.ws.run_table(keys, self.table.t)
            sl.rows = sl.ws.rows_u
        else:
            sl.ws.run(keys, False)
            self.table.t.probe_into(sl.ws.uniq_h[:L], sl.ws.u_count, sl.rows)
        self._prepared[keys.data_ptr()] = (sl, L)
        self._keep_keys(keys)

    def _keep_keys(self, keys: torch.Tensor):
        """Prepared pulls are looked up by the key buffer's address: keep that
        buffer's storage alive while its entry exists, so a later batch can
        never get the same address and pick up this batch's prepared state
        (ADVICE r4).  Dropped with the entries (clear_prefetch)."""
        self._prepared_keep[keys.data_ptr()] = keys.untyped_storage()

    def can_prefetch_pull(self) -> bool:
        if self.sharded:
            # the whole sharded pull (dedup, key / answer exchanges on the IPC
            # meshes, owner probe + gather, pooling) ahead of its step: IPC
            # meshes only (capturable, no RCCL inside the graphs), fixed keys
            return (self.is_gpu and self.xmesh is not None and self.codec is None and self.dedup
                    and not (self.auto_insert and not self.test_mode) and len(self._slots) >= 2)
        return self.can_prefetch() and self.table_dedup and self.codec is None

    def prefetch_pull(self, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int, sp: "SeqpoolParams",
                      dense: Optional[torch.Tensor] = None, slot: int = 0) -> bool:
        """Dedup + probe AND the fused seqpool + CVM (+ dense columns) of a
        batch ahead of its training step, into pull slot ``slot`` and its
        persistent output buffer.  Issued after the previous step's sparse
        push (the pooled values must include that update) on the compute
        stream, it runs under the previous step's dW GEMM; the batch's own
        pull then returns the buffer with no launch at all.  False when the
        engine cannot prepare pulls (sharded, codec rows, auto-insert)."""
        if self.sharded:
            return self._prefetch_pull_sharded(keys, lod, B, S, sp, dense, slot)
        if not self.prefetch_dedup(keys, slot):
            return False
        return self.prefetch_pool(keys, lod, B, S, sp, dense, slot)

    def _prefetch_pull_sharded(self, keys, lod, B, S, sp, dense, slot) -> bool:
        """Sharded prefetch_pull: the complete pull of the next batch into pull
        slot ``slot`` -- sender dedup, key exchange, owner probe + gather,
        answer exchange, fused seqpool/CVM into the slot's persistent output.
        Issued after this step's push (and its owner-side update) in stream
        order on every rank, so every owner answers with the updated rows."""
        if not self.can_prefetch_pull():
            return False
        keys = keys.reshape(-1)
        L = keys.numel()
        assert L <= self.max_keys
        sl = self._slots[slot % len(self._slots)]
        sl.gen += 1
        st = self._pull_into_slot(sl, keys, lod, B, S, fill_occ=False)
        self._pool_sharded(sl, st, keys, lod, B, S, sp, dense)
        return True

    def _pool_sharded(self, sl: _PullSlot, st: PullState, keys, lod, B, S, sp, dense):
        """Fused seqpool/CVM of a prefetched sharded pull into the slot's
        persistent output; the pull state is kept for the batch's own step."""
        L = keys.numel()
        Eo = sp.out_width(self.E)
        Dd = 0 if dense is None else int(dense.shape[1])
        shape = (B, S * Eo + Dd)
        sl.pooled_out(shape, self.device)
        self._hip.seqpool_cvm_fwd(sl.resp_back, sl.send_index, sl.ws.uid, lod, S, B, self.E, sl.pre_out, 0,
                                  sp.use_cvm, sp.cvm_offset, sp.clk_filter, sp.pad_value, sp.need_filter,
                                  sp.show_coeff, sp.clk_coeff, sp.threshold, sp.quant_ratio,
                                  sp.embed_threshold_filter, sp.embed_threshold,
                                  sp.embed_thres_size if not sp.use_cvm else 0,
                                  _dense_rows(dense) if dense is not None else None, S * Eo,
                                  occ_slot=sl.occ_slot, occ_ins=sl.occ_ins)
        self._prepared[keys.data_ptr()] = (sl, L, st)
        self._prepared_out[keys.data_ptr()] = sl.pre_out
        self._keep_keys(keys)

    def prefetch_dedup(self, keys: torch.Tensor, slot: int = 0) -> bool:
        """The key half of prefetch_pull (table dedup + probe into the slot):
        depends on the keys only, so it may run on a side stream beside the
        previous step's sparse push."""
        if not self.can_prefetch_pull():
            return False
        assert keys.numel() <= self.max_keys
        sl = self._slots[slot % len(self._slots)]
        if self.sharded:
            # the sender dedup only (keys -> uniques, per-owner counts); the
            # pack, both exchanges and the pooling follow in prefetch_pool
            self._hash_dedup(sl, keys.reshape(-1))
            if self.xmesh is not None and _early_key_exchange():
                # the key exchange too: it reads only this batch's keys, so it
                # runs here, off the step's sparse chain (the owners' probe +
                # gather and the answer exchange wait for the push: prefetch_pool)
                self._key_exchange(sl)
                sl.keys_exchanged = True
            return True
        if self._finish_side():
            # the pooling needs only the probe + rank launch (rows_occ); the
            # run starts + scatter (uid / perm / counters) are the next push's:
            # they run on a side stream beside the pooling, joined with the
            # step's other side work (parallel.dense grad producers)
            from ..parallel.dense import add_grad_producer

            sl.ws.run_table(keys, self.table.t, False, False, 1)
            cur = torch.cuda.current_stream(self.device)
            side = side_stream(self.device, "td_finish")
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                sl.ws.run_table(keys, self.table.t, False, False, 2)
            add_grad_producer(side)
        else:
            sl.ws.run_table(keys, self.table.t, False, self._fuse_scatter())
        sl.rows = sl.ws.rows_u
        return True

    def _finish_side(self) -> bool:
        """PBX_TD_FINISH_SIDE=1: the prefetched table dedup's run starts +
        scatter on a side stream beside the pooling (not with the fused
        scatter, which the pooling launch itself performs)."""
        return os.environ.get("PBX_TD_FINISH_SIDE", "0") == "1" and not self._fuse_scatter()

    def _fuse_scatter(self) -> bool:
        """Leave the table dedup's scatter to the prefetched pooling launch
        (PBX_FUSED_SCATTER=1): one launch less on the step's sparse chain."""
        return (self.seqpool_rows_occ and self.codec is None and self.E in (11, 12, 19, 35)
                and os.environ.get("PBX_FUSED_SCATTER", "0") == "1")

    def prefetch_pool(self, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int, sp: "SeqpoolParams",
                      dense: Optional[torch.Tensor] = None, slot: int = 0) -> bool:
        """The value half of prefetch_pull: the fused seqpool of the slot's
        deduplicated batch into its persistent output (after prefetch_dedup
        and after every push the values must include, in stream order)."""
        if not self.can_prefetch_pull():
            return False
        L = keys.numel()
        sl = self._slots[slot % len(self._slots)]
        if self.sharded:
            sl.gen += 1
            st = self._sharded_after_dedup(sl, L, lod, B, S)
            self._pool_sharded(sl, st, keys, lod, B, S, sp, dense)
            return True
        ws = sl.ws
        Eo = sp.out_width(self.E)
        Dd = 0 if dense is None else int(dense.shape[1])
        shape = (B, S * Eo + Dd)
        sl.pooled_out(shape, self.device)
        if self.seqpool_rows_occ:
            src_index, uid = ws.rows_occ[:L], None
        else:
            src_index, uid = ws.rows_u, ws.uid
        self._hip.seqpool_cvm_fwd(self.table.values, src_index, uid, lod, S, B, self.E, sl.pre_out, 0, sp.use_cvm,
                                  sp.cvm_offset, sp.clk_filter, sp.pad_value, sp.need_filter, sp.show_coeff,
                                  sp.clk_coeff, sp.threshold, sp.quant_ratio, sp.embed_threshold_filter,
                                  sp.embed_threshold, sp.embed_thres_size if not sp.use_cvm else 0,
                                  _dense_rows(dense) if dense is not None else None, S * Eo,
                                  occ_slot=sl.occ_slot, occ_ins=sl.occ_ins, scatter_ws=ws)
        self._prepared[keys.data_ptr()] = (sl, L)
        self._prepared_out[keys.data_ptr()] = sl.pre_out
        self._keep_keys(keys)
        return True

    def prepared_output(self, keys: torch.Tensor) -> Optional[torch.Tensor]:
        """The pooled output a prefetch_pull left for this key buffer (or None)."""
        return self._prepared_out.get(keys.data_ptr()) if self.is_gpu else None

    def clear_prefetch(self, reset_rows: bool = False):
        """Forget the prepared pulls.  reset_rows: also hand every pull slot's
        occurrence rows back all -1 now (eagerly, so a step captured next
        does not carry the clean-up; SparseEngine._pull_split)."""
        self._prepared.clear()
        self._prepared_out.clear()
        getattr(self, "_prepared_keep", {}).clear()
        if reset_rows and self.is_gpu:
            for sl in getattr(self, "_slots", []):
                if getattr(sl.ws, "rows_occ_dirty", False):
                    sl.ws.clean_rows_occ()

    def ensure_pull_ring(self, n: int):
        """At least ``n`` pull slots (the pipelined front keys slots by batch
        buffer: n_buffers x steps per graph).  Not inside a graph capture."""
        if self.is_gpu and len(self._slots) < n:
            self._slots += [_PullSlot(self) for _ in range(n - len(self._slots))]

    def reset_pull_ring(self):
        """Fresh pull slots (dedup workspaces, occurrence maps, pooled
        outputs) and zeroed push scratch -- what a new training program over
        the same table starts from (bench.py: each same-run measurement)."""
        if not self.is_gpu:
            return
        self.clear_prefetch()
        self._pending_dedup = None
        n = len(self._slots)
        self._slots = [_PullSlot(self) for _ in range(n)]
        self._next_slot = 0
        self._cur = self._slots[0]
        if getattr(self, "push_acc", None) is not None:
            self.push_acc.zero_()
            self.push_inc = _push_run_scratch(self.max_keys, self.device)

    def _take_slot(self) -> _PullSlot:
        sl = self._slots[self._next_slot % len(self._slots)]
        self._next_slot += 1
        sl.gen += 1
        self._cur = sl
        return sl

    def _check_slot(self, st: PullState) -> _PullSlot:
        sl = st.slot
        if sl is None or sl.gen != st.gen:
            raise RuntimeError(
                f"stale pull state: its buffers were reused by a later pull (more than {len(self._slots)} pulls "
                "outstanding before their push); construct the SparseEngine with a larger pull_ring")
        return sl

    def _pull_common(self, keys, lod, B, S, fill_occ: bool = True) -> PullState:
        h = self._hip
        L = keys.numel()
        assert L <= self.max_keys, f"batch has {L} keys > engine max_keys {self.max_keys}"
        pre = self._prepared.pop(keys.data_ptr(), None) if self._prepared else None
        if pre is not None and pre[1] == L and self.sharded and len(pre) > 2:
            # prefetch_pull ran the whole sharded pull (exchanges included)
            # into this slot: its state is the pull state
            st = pre[2]
            self._cur = pre[0]
            return st
        if pre is not None and pre[1] == L and not self.sharded:
            sl = pre[0]
            sl.gen += 1
            self._cur = sl
            if fill_occ:
                h.fill_occurrence(lod, S, B, sl.occ_slot, sl.occ_ins)
            ws = sl.ws
            st = PullState(B=B, S=S, L=L, lod=lod, uid=ws.uid, perm=ws.perm, counts=ws.u_count, slot=sl,
                           gen=sl.gen)
            st.rows = sl.rows[:L]
            return st
        return self._pull_into_slot(self._take_slot(), keys, lod, B, S, fill_occ)

    def _pull_into_slot(self, sl: _PullSlot, keys, lod, B, S, fill_occ: bool) -> PullState:
        h = self._hip
        L = keys.numel()
        ws = sl.ws
        if self.table_dedup:
            ws.run_table(keys, self.table.t)
            if fill_occ:
                h.fill_occurrence(lod, S, B, sl.occ_slot, sl.occ_ins)
            st = PullState(B=B, S=S, L=L, lod=lod, uid=ws.uid, perm=ws.perm, counts=ws.u_count, slot=sl,
                           gen=sl.gen)
            st.rows = ws.rows_u[:L]
            st.extra["rows_occ"] = ws.rows_occ[:L]
            if self.auto_insert and not self.test_mode:
                miss = (ws.rows_occ[:L] < 0) & (keys.reshape(-1) != -1)
                if bool(miss.any()):
                    self.table.insert_mixed(torch.unique(ref.mix64(keys.reshape(-1)[miss])), self.cfg.sgd)
                    ws.run_table(keys, self.table.t)
            return st
        self._hash_dedup(sl, keys)
        if fill_occ:
            h.fill_occurrence(lod, S, B, sl.occ_slot, sl.occ_ins)
        if not self.sharded:
            st = PullState(B=B, S=S, L=L, lod=lod, uid=ws.uid, perm=ws.perm, counts=ws.u_count, slot=sl,
                           gen=sl.gen)
            st.rows = self.table.probe(ws.uniq_h[:L], ws.u_count)
            if self.auto_insert and not self.test_mode:
                self._auto_insert(st, L)
            return st
        return self._sharded_after_dedup(sl, L, lod, B, S)

    def _hash_dedup(self, sl: _PullSlot, keys):
        # IPC exchange: the shard pack's per-owner counters are zeroed by the
        # dedup's first launch (no fill launches of their own)
        ipc = self.sharded and self.xmesh is not None
        sl.ws.run(keys, False, sl.ocnt if ipc else None)

    def _fused_exchanges(self) -> bool:
        return (self.xmesh is not None and _pack_exchange() and hasattr(self.xmesh[0].comm, "pack_exchange")
                and hasattr(self.table.t, "answer_exchange"))

    def _key_exchange(self, sl: _PullSlot):
        """Sender half of a sharded pull after its dedup: pack the unique keys
        per owner and exchange them (the keys only -- no table access, so it
        may run ahead of the previous batch's push: prefetch_dedup)."""
        ws = sl.ws
        ipc = self.xmesh is not None
        if self._fused_exchanges():
            # the pack inside the key exchange's put phase: the dedup output
            # goes straight to the owners' inboxes (no send buffer)
            self.xmesh[0].pack_exchange(ws.uniq_h, ws.u_count, self.C, sl.send_index, sl.ocnt, self.overflow,
                                        sl.recv.view(self.world, -1), sl.rcnt)
            return
        self._hip.shard_pack_hash(ws.uniq_h, ws.u_count, self.world, self.C, sl.send, sl.send_index, sl.ocnt,
                                  self.overflow, ipc)
        if ipc:
            # only the valid keys of each peer slot travel; the receiver
            # fills the rest of its slots with -1 (padding for the dedup)
            self.xmesh[0].exchange(sl.send.view(self.world, -1), sl.recv.view(self.world, -1), sl.ocnt, 8, True,
                                   sl.rcnt)
        else:
            self.comm.all_to_all_single(sl.recv, sl.send)

    def _sharded_after_dedup(self, sl: _PullSlot, L: int, lod, B: int, S: int) -> PullState:
        """Sharded pull after the sender dedup: pack per owner, key exchange
        (unless prefetch_dedup already ran them), owner probe + gather, answer
        exchange."""
        fused = self._fused_exchanges()
        st = PullState(B=B, S=S, L=L, lod=lod, uid=sl.ws.uid, perm=sl.ws.perm, counts=sl.ws.u_count, slot=sl,
                       gen=sl.gen)
        if sl.keys_exchanged:
            sl.keys_exchanged = False
        else:
            self._key_exchange(sl)
        if self.codec is None:
            # owner answers in one launch: probe + record copy per received
            # key, no dedup (a key asked by several peers is read twice)
            rows_r = sl.rows_recv
            if fused and not (self.auto_insert and not self.test_mode):
                # ... straight into the askers' inboxes inside the answer
                # exchange (no answer buffer in between)
                m = self.xmesh[1]
                with m._serial("answer_exchange"):
                    self.table.t.answer_exchange(m.comm.peers_ptr(), m.comm.blocks(), sl.recv, sl.rcnt, self.C,
                                                 rows_r, sl.resp_back)
                st.send_index = sl.send_index[:L]
                st.rows_r = rows_r
                return st
            self.table.t.probe_gather(sl.recv, rows_r, sl.resp)
            if self.auto_insert and not self.test_mode:
                miss = (rows_r < 0) & (sl.recv != -1)
                if bool(miss.any()):
                    self.table.insert_mixed(torch.unique(sl.recv[miss]), self.cfg.sgd)
                    self.table.t.probe_gather(sl.recv, rows_r, sl.resp)
            return self._answer(sl, st, L, rows_r)
        sl.ws_r.run(sl.recv, True)
        rows_r = self.table.probe(sl.ws_r.uniq_h, sl.ws_r.u_count)
        if self.auto_insert and not self.test_mode:
            miss = (rows_r[: int(sl.ws_r.u_count[0].item())] < 0)
            if bool(miss.any()):
                U = int(sl.ws_r.u_count[0].item())
                self.table.insert_mixed(sl.ws_r.uniq_h[:U][miss], self.cfg.sgd)
                rows_r = self.table.probe(sl.ws_r.uniq_h, sl.ws_r.u_count)
        # owner answers straight from the table rows (no intermediate pull buffer)
        self.table.t.codec_pull(self.codec.native(), rows_r, sl.ws_r.uid, None, sl.resp.shape[0], sl.resp)
        return self._answer(sl, st, L, rows_r)

    def _answer(self, sl: _PullSlot, st: PullState, L: int, rows_r: torch.Tensor) -> PullState:
        if self.xmesh is not None:
            # answers: as many rows to each peer as it sent keys
            self.xmesh[1].exchange(sl.resp.view(self.world, -1), sl.resp_back.view(self.world, -1), sl.rcnt,
                                   self.P * 4, False, None)
        else:
            self.comm.all_to_all_single(sl.resp_back, sl.resp)
        st.send_index = sl.send_index[:L]
        st.rows_r = rows_r
        return st

    def _auto_insert(self, st: PullState, L: int):
        ws = st.slot.ws
        U = int(ws.u_count[0].item())
        miss = st.rows[:U] < 0
        if bool(miss.any()):
            self.table.insert_mixed(ws.uniq_h[:U][miss], self.cfg.sgd)
            st.rows = self.table.probe(ws.uniq_h[:L], ws.u_count)

    # ------------------------------------------------------------------ push
    def push_seqpool_cvm(self, st: PullState, dout: torch.Tensor, cvm: torch.Tensor, col_offset: int,
                         sp: SeqpoolParams, bs_scale: float):
        """Backward of the fused op = push_box_sparse with fused Adagrad."""
        if self.test_mode:
            return
        if not self.is_gpu:
            return self._cpu_push(st, dout, cvm, col_offset, sp, bs_scale)
        sl = self._check_slot(st)
        if "dedup_event" in st.extra:
            self._join_dedup(st)
        ws = sl.ws
        h = self._hip
        L = st.L
        dout = dout.contiguous()
        ets = 0 if sp.use_cvm else sp.embed_thres_size
        if st.extra.get("nodedup"):
            self._seed += 1
            if not self.table.t.push_occ(dout, col_offset, cvm.contiguous(), sp.use_cvm, sp.clk_filter, self.E,
                                         sl.occ_slot, sl.occ_ins, self._slot_ids(st.S), st.rows, self.push_acc_occ,
                                         float(bs_scale), self._sgd_native, self._seed, ets):
                raise RuntimeError("no-dedup push needs cvm_offset 2 with a [B, 2] cvm (use the dedup path)")
            return
        if not self.sharded:
            if sp.cvm_offset == 2 and cvm.shape[1] == 2 and self.codec is None:
                self._seed += 1
                if self.table.t.push_merge_apply(dout, col_offset, cvm.contiguous(), sp.use_cvm, sp.clk_filter, self.E,
                                                 ws.perm[:L], ws.uid, sl.occ_slot, sl.occ_ins,
                                                 self._slot_ids(st.S), ws.u_count[1:], self.push_acc,
                                                 self.push_inc, float(bs_scale), st.rows, self._sgd_native,
                                                 self._seed, ets):
                    return
                self._seed -= 1
            push = self.push_buf
            push[:L].zero_()
            h.push_merge(dout, col_offset, cvm.contiguous(), sp.cvm_offset, sp.use_cvm, sp.clk_filter, self.E,
                         ws.perm[:L], ws.uid, sl.occ_slot, sl.occ_ins, self._slot_ids(st.S),
                         ws.u_count[1:], push[:L], None, float(bs_scale), self.dim, ets)
            self._seed += 1
            self._update_rows(st.rows, push[:L], ws.u_count)
            return
        if (sp.cvm_offset == 2 and cvm.shape[1] == 2 and self.codec is None
                and h.push_merge_send(dout, col_offset, cvm.contiguous(), sp.use_cvm, sp.clk_filter, self.E,
                                      ws.perm[:L], ws.uid, sl.occ_slot, sl.occ_ins, self._slot_ids(st.S),
                                      ws.u_count[1:], self.push_acc, self.push_inc, self.push_send, st.send_index,
                                      float(bs_scale), self.dim, ets)):
            # merged records went straight into their send slots
            self._owner_update(sl, st.rows_r, self._push_exchange(sl))
            return
        self.push_send.zero_()
        h.push_merge(dout, col_offset, cvm.contiguous(), sp.cvm_offset, sp.use_cvm, sp.clk_filter, self.E,
                     ws.perm[:L], ws.uid, sl.occ_slot, sl.occ_ins, self._slot_ids(st.S),
                     ws.u_count[1:], self.push_send, st.send_index, float(bs_scale), self.dim, ets)
        self._owner_update(sl, st.rows_r, self._push_exchange(sl))

    def _push_exchange(self, sl: _PullSlot) -> torch.Tensor:
        """Merged gradient records to the key owners (same per-peer counts as
        the keys of this pull)."""
        if self.xmesh is not None:
            self.xmesh[2].exchange(self.push_send.view(self.world, -1), self.push_recv.view(self.world, -1), sl.ocnt,
                                   self.Q * 4, False, None)
        else:
            self.comm.all_to_all_single(self.push_recv, self.push_send)
        return self.push_recv

    def _owner_update(self, sl: _PullSlot, rows_r: torch.Tensor, recv: torch.Tensor):
        """Owner side of the push: each key got at most one merged record per
        sender.  Plain rows: rows_r holds the row of every received entry;
        the entries of one row elect a leader that sums the others' records
        and applies sparse Adagrad (two launches, no dedup).  Codec rows (or
        a dim without the vector kernels): dedup the received keys, merge,
        then the codec / generic update."""
        self._seed += 1
        ws = sl.ws_r
        if self.codec is None:
            if self.table.t.owner_push(rows_r, recv, self._sgd_native, self._seed):
                return
            ws.run(sl.recv, True)
            rows_r = self.table.probe(ws.uniq_h, ws.u_count)
        self.push_merged.zero_()
        self._hip.push_merge_records(recv, ws.perm, ws.uid, ws.u_count[1:], self.xdim, self.push_merged)
        self._update_rows(rows_r, self.push_merged, ws.u_count)

    def _update_rows(self, rows: torch.Tensor, push: torch.Tensor, n_dev: torch.Tensor):
        """Apply merged per-unique push records to the table rows (sparse
        Adagrad, or the feature-type codec's rule)."""
        if self.codec is not None:
            self.table.t.codec_update(self.codec.native(), rows, push, n_dev, self._sgd_native, self._seed)
        else:
            self.table.t.push_adagrad(rows, push, n_dev, self._sgd_native, self._seed)

    def _slot_ids(self, S: int) -> torch.Tensor:
        if self.slot_ids.numel() < S:
            self.slot_ids = torch.arange(S, dtype=torch.float32, device=self.device)
        return self.slot_ids

    GUARD_BITS = {1: "push: table row outside the table", 2: "dedup: row without a unique id of its batch",
                  4: "dedup: perm slot outside the batch", 8: "push: occurrence / unique id outside the batch",
                  16: "seqpool: lod occurrence outside the occurrence buffers",
                  32: "seqpool: unique id outside the record index", 64: "seqpool: record outside the pulled source"}

    def check_guards(self):
        """Raise if a kernel met an out-of-range index (skipped, not followed:
        TableDev::err).  A device read: call outside graph captures."""
        if not self.is_gpu:
            return
        bits = int(self.table.t.error_bits())
        dev = self._guard_dev
        bits |= int(self._hip.guard_bits(dev))  # the seqpool's (process-wide word)
        if bits:
            self.table.t.clear_error()
            self._hip.clear_guard_bits(dev)
            what = "; ".join(v for b, v in self.GUARD_BITS.items() if bits & b)
            raise RuntimeError(f"sparse engine index guard tripped (bits {bits:#x}): {what}")

    def check_overflow(self) -> bool:
        self.check_exchange()
        self.check_guards()
        if self.sharded and self.is_gpu:
            return bool(self.overflow.item())
        return False

    # ------------------------------------------------------------------ unfused pull (pull_box_sparse)
    def pull_records(self, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int, with_expand: bool = False):
        """pull_box_sparse: per-occurrence pull records [L, 3+D] (box_wrapper.cu:74-143);
        with_expand: [L, 3+D+De] including the expand block (pull_box_extended_sparse)."""
        L = keys.numel()
        W = 3 + self.xdim if with_expand else self.E
        if not self.is_gpu:
            uniq, uid = ref.dedup(keys)
            rows = self.table.probe(uniq)
            pulled = self.table.gather_pull(rows, self.P)
            st = PullState(B=B, S=S, L=L, lod=lod, uid=uid, rows=rows)
            st.extra["uniq"] = uniq
            recs = torch.where((keys != -1).unsqueeze(1), pulled[uid.long().clamp(min=0)], torch.zeros(1))
            return recs[:, : self.E], st
        st = self._pull_common(keys, lod, B, S)
        sl = st.slot
        if not self.sharded:
            if self.codec is not None:
                pulled = torch.empty(L, self.P, device=self.device)
                self.table.t.codec_pull(self.codec.native(), st.rows, None, sl.ws.u_count, L, pulled)
            else:
                pulled = self.table.t.gather_pull(st.rows, sl.ws.u_count, self.P)
            recs = torch.empty(L, self.P, device=self.device)
            self._hip.gather_by_uid(pulled, sl.ws.uid[:L], recs, self.P)
        else:
            # resp_back rows indexed by send_index[uid]
            idx = sl.send_index[:L][sl.ws.uid[:L].long().clamp(min=0)]
            ok = (sl.ws.uid[:L] >= 0) & (idx >= 0)
            recs = torch.where(ok.unsqueeze(1), sl.resp_back[idx.clamp(min=0)], torch.zeros((), device=self.device))
        if with_expand and self.codec is not None and self.codec.kind == 3:
            W += 1  # variable: [show, click, embed_w, block[max(D, De)], size]
        return recs[:, :W], st

    def push_records(self, st: PullState, grads: torch.Tensor, cvm_cols: int, bs_scale: float,
                     slot_of_occ: Optional[torch.Tensor] = None):
        """push_box_sparse from per-occurrence grads [L, 3+D] of the pull output:
        columns < cvm_cols are show/click statistics, the rest are scaled by
        -bs (box_wrapper.cu:344-475)."""
        if self.test_mode:
            return
        L = st.L
        D = min(self.xdim, grads.shape[1] - 3) if self.is_gpu else self.dim
        g = grads.float()
        rec = torch.zeros(L, self.Q, device=grads.device)
        if slot_of_occ is None:
            slot_of_occ, _ = ref.occurrence_map(st.lod.cpu(), st.S, st.B)
            slot_of_occ = slot_of_occ.to(grads.device)
        rec[:, 0] = self._slot_ids(st.S)[slot_of_occ.long()]
        rec[:, 1] = g[:, 0]
        rec[:, 2] = g[:, 1]
        rec[:, 3:4 + D] = g[:, 2:3 + D] * (-bs_scale)
        if not self.is_gpu:
            U = st.extra["uniq"].numel()
            merged = torch.zeros(U, self.Q)
            ok = st.uid >= 0
            merged.index_add_(0, st.uid[ok].long(), rec[ok])
            merged[:, 0] = 0
            merged[st.uid[ok].long(), 0] = rec[ok, 0]
            self.table.push_adagrad(st.rows, merged, self.cfg.sgd)
            return
        sl = self._check_slot(st)
        ws = sl.ws
        h = self._hip
        if not self.sharded:
            push = self.push_buf
            push[:L].zero_()
            h.push_merge_records(rec, ws.perm[:L], ws.uid, ws.u_count[1:], self.xdim, push[:L])
            self._seed += 1
            self._update_rows(st.rows, push[:L], ws.u_count)
            return
        # merge locally per unique into the owner send layout, then exchange
        U_cap = L
        merged = torch.zeros(U_cap, self.Q, device=self.device)
        h.push_merge_records(rec, ws.perm[:L], ws.uid, ws.u_count[1:], self.xdim, merged)
        self.push_send.zero_()
        idx = st.send_index
        ok = idx >= 0
        self.push_send[idx[ok]] = merged[ok]
        self._owner_update(sl, st.rows_r, self._push_exchange(sl))

    # ------------------------------------------------------------------ CPU path
    def _cpu_pull_seqpool(self, keys, lod, B, S, out, col_offset, sp: SeqpoolParams) -> PullState:
        L = keys.numel()
        valid = keys != -1
        uniq, uid = ref.dedup(keys[valid])
        full_uid = torch.full((L,), -1, dtype=torch.int32)
        full_uid[valid] = uid
        if self.sharded:
            return self._cpu_pull_sharded(keys, lod, B, S, out, col_offset, sp, uniq, full_uid)
        rows = self.table.probe(uniq)
        if self.auto_insert and not self.test_mode and bool((rows < 0).any()):
            self.table.insert_mixed(uniq[rows < 0], self.cfg.sgd)
            rows = self.table.probe(uniq)
        pulled = self.table.gather_pull(rows, self.P)
        y = ref.seqpool_cvm(pulled, full_uid, lod, S, B, self.E, sp.use_cvm, sp.cvm_offset, sp.clk_filter,
                            sp.pad_value, sp.need_filter, sp.show_coeff, sp.clk_coeff, sp.threshold,
                            sp.quant_ratio, sp.embed_threshold_filter, sp.embed_threshold, sp.embed_thres_size)
        out[:, col_offset:col_offset + y.shape[1]] = y
        st = PullState(B=B, S=S, L=L, lod=lod, uid=full_uid, rows=rows)
        st.extra["U"] = uniq.numel()
        return st

    def _cpu_pull_sharded(self, keys, lod, B, S, out, col_offset, sp, uniq, full_uid) -> PullState:
        W = self.world
        owner = ref.owner_of(uniq, W)
        order = torch.argsort(owner, stable=True)
        uniq_o = uniq[order]
        counts = torch.bincount(owner, minlength=W)
        in_counts = torch.empty_like(counts)
        self.comm.all_to_all_single(in_counts, counts)
        recv = torch.empty(int(in_counts.sum()), dtype=torch.int64)
        self.comm.all_to_all_single(recv, uniq_o, in_counts.tolist(), counts.tolist())
        rows_r = self.table.probe(recv)
        if self.auto_insert and not self.test_mode and bool((rows_r < 0).any()):
            self.table.insert_mixed(torch.unique(recv[rows_r < 0]), self.cfg.sgd)
            rows_r = self.table.probe(recv)
        pulled_r = self.table.gather_pull(rows_r, self.P)
        back = torch.empty(uniq.numel(), self.P)
        self.comm.all_to_all_single(back, pulled_r, counts.tolist(), in_counts.tolist())
        pulled = torch.empty_like(back)
        pulled[order] = back
        y = ref.seqpool_cvm(pulled, full_uid, lod, S, B, self.E, sp.use_cvm, sp.cvm_offset, sp.clk_filter,
                            sp.pad_value, sp.need_filter, sp.show_coeff, sp.clk_coeff, sp.threshold,
                            sp.quant_ratio, sp.embed_threshold_filter, sp.embed_threshold, sp.embed_thres_size)
        out[:, col_offset:col_offset + y.shape[1]] = y
        st = PullState(B=B, S=S, L=keys.numel(), lod=lod, uid=full_uid)
        st.extra.update(U=uniq.numel(), order=order, counts=counts, in_counts=in_counts, rows_r=rows_r,
                        recv=recv)
        return st

    def _cpu_push(self, st: PullState, dout, cvm, col_offset, sp: SeqpoolParams, bs_scale):
        U = st.extra["U"]
        push = ref.push_merge(dout, cvm, st.uid, st.lod, st.S, st.B, U, self.dim, self._slot_ids(st.S), bs_scale,
                              sp.use_cvm, sp.clk_filter, col_offset, sp.cvm_offset, sp.embed_thres_size)
        if not self.sharded:
            self.table.push_adagrad(st.rows, push, self.cfg.sgd)
            return
        e = st.extra
        send = push[e["order"]]
        recv = torch.empty(int(e["in_counts"].sum()), push.shape[1])
        self.comm.all_to_all_single(recv, send, e["in_counts"].tolist(), e["counts"].tolist())
        # merge duplicates from different senders, then update
        uq, inv = torch.unique(e["recv"], return_inverse=True)
        merged = torch.zeros(uq.numel(), push.shape[1])
        merged.index_add_(0, inv, recv)
        merged[inv, 0] = recv[:, 0]
        rows = self.table.probe(uq)
        self.table.push_adagrad(rows, merged, self.cfg.sgd)
