"""Tiered sparse store: HBM working set <- host tier <- SSD tier.

BoxPS trains a pass out of HBM while the next pass's feature values are
staged from host memory / SSD and the previous pass's are written back
(FeedPass / BeginPass / EndPass, box_wrapper.h:1142-1183,
box_wrapper.cc:120-210).  MI355X design:

* The live GPU table never moves (captured HIP graphs hold its addresses).
  The next pass is staged into a second, identically shaped GPU table on a
  side stream; ``activate`` (BeginPass) copies the rows the two passes share
  from the live table into the staged one (their newest values) and then
  copies the staged table over the live one device-to-device (~1 ms per
  10 GB of HBM3E).
* Staging runs in a background thread: host-tier probe / SSD reads /
  gather into a pinned buffer are native and GIL-free (csrc/host/
  tier_store.cc), then one H2D copy and the GPU insert + assign.
* Feature-type codecs (int16, SparseAdam, expand, variable) are tiered in
  their canonical fp32 layout (``FeatureCodec.decode`` / ``encode``): the
  host and SSD tiers never see the packed device encoding.
* EndPass exports the live table (a device copy) and a background thread
  moves it D2H into the host tier and spills to the log-structured SSD tier
  -- overlapped with the next pass's training.  Two spill rules: rows unseen
  for ``spill_unseen`` days, and a host-tier row cap (``host_cap_rows``):
  every host row carries the id of the pass that last wrote it, and the rows
  of the oldest passes move to SSD until the cap holds.  Staging of pass n+2
  waits for write-back of pass n, so every staged value is current.
"""
from __future__ import annotations

import threading
import time
from typing import Optional, Tuple

import torch

from .. import _native
from .config import ShrinkConfig, SparseSGDConfig, row_layout


class HostTable:
    """CpuSparseTable-compatible facade over the native HostTier."""

    def __init__(self, dim: int, threads: int = 16, chunk_rows: int = 1 << 20, stride: Optional[int] = None):
        self.dim = dim
        self.layout = row_layout(dim)
        self.stride = int(stride or self.layout["stride"])
        self.device = torch.device("cpu")
        self._native = _native.host().HostTier(self.stride, threads, chunk_rows)

    def probe(self, h: torch.Tensor, n_dev=None) -> torch.Tensor:
        return self._native.probe(h.reshape(-1).cpu())

    def insert_mixed(self, h: torch.Tensor, sgd: SparseSGDConfig, init_embedx: bool = False, n_dev=None) -> int:
        h = h.reshape(-1).cpu()
        h = h[h != -1]
        if h.numel() == 0:
            return 0
        before = self._native.probe(h)
        rows, fresh = self._native.insert(h)
        new = before < 0
        if bool(new.any()) and (sgd.initial_range > 0 or init_embedx):
            v = torch.zeros(int(new.sum()), self.stride)
            if sgd.initial_range > 0:
                v[:, 2] = (torch.rand(v.shape[0]) * 2 - 1) * sgd.initial_range
            if init_embedx:
                v[:, 3:3 + self.dim] = torch.rand(v.shape[0], self.dim) * sgd.mf_initial_range
                v[:, self.layout["mf_size"]] = 1
            self._native.scatter(rows[new], v)
        return 0

    def assign(self, h: torch.Tensor, vals: torch.Tensor):
        rows = self.probe(h)
        self._native.scatter(rows, vals.cpu().float())

    def stamp_keys(self, h: torch.Tensor, epoch: int):
        """Pass stamp of the rows of h (the spill_oldest order)."""
        self._native.stamp(self.probe(h), int(epoch))

    def read(self, h: torch.Tensor) -> torch.Tensor:
        rows = self.probe(h)
        out = torch.empty(rows.numel(), self.stride)
        self._native.gather(rows, out)
        return out

    def export(self, with_values: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        k, v = self._native.export_all()
        return k, (v if with_values else None)

    def erase(self, h: torch.Tensor) -> int:
        return int(self._native.erase(h.reshape(-1).cpu()))

    def size(self) -> int:
        return int(self._native.size())

    @property
    def capacity(self) -> int:
        return self.size()

    def memory_bytes(self) -> int:
        return int(self._native.memory_bytes())

    def shrink(self, cfg: ShrinkConfig) -> int:
        """Decay show/click, age, delete (ctr_accessor.cc:63-80) over the host
        tier, natively and in place (HostTier::shrink: parallel over shards)."""
        return int(self._native.shrink(float(cfg.show_click_decay_rate), int(self.layout["unseen_days"]),
                                       float(cfg.nonclk_coeff), float(cfg.clk_coeff), float(cfg.delete_threshold),
                                       float(cfg.delete_after_unseen_days)))

    def clear(self):
        self._native.clear()


class SsdTier:
    """Facade over the native log-structured SsdLog (csrc/host/tier_store.cc)."""

    def __init__(self, path: str, stride: int, segment_bytes: int = 64 << 20):
        import os

        self.path = path
        self.stride = stride
        os.makedirs(path, exist_ok=True)
        self._native = _native.host().SsdLog(path, stride, int(segment_bytes))

    def __len__(self):
        return int(self._native.size())

    def put(self, h: torch.Tensor, v: torch.Tensor):
        if h.numel():
            self._native.put(h.reshape(-1).cpu(), v.cpu().float())

    def get(self, h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        return self._native.get(h.reshape(-1).cpu())

    def delete(self, h: torch.Tensor):
        if h.numel():
            self._native.erase(h.reshape(-1).cpu())

    def compact(self, min_live: float = 0.5) -> int:
        return int(self._native.compact(min_live))

    def keys(self) -> torch.Tensor:
        return self._native.keys()

    def disk_bytes(self) -> int:
        return int(self._native.disk_bytes())

    @property
    def direct_io(self) -> bool:
        return bool(self._native.direct_io())


class TierView:
    """The tiered sparse model as one table: the host tier plus the SSD log.

    Every key lives in exactly one tier (staging and ``promote`` move SSD rows
    to the host, spills move host rows to SSD, write-back drops the SSD copy
    of a key that re-enters the host), so BoxWrapper's model IO and shrink see
    the whole table -- SaveBase / SaveDelta / load / ShrinkTable over every
    feature, as the reference PS does (box_wrapper.cc:1286-1318,
    box_wrapper.h:638; accessor rules ctr_accessor.cc:63-170).

    * saves stream natively (``save_tiers``, csrc/host/tier_save.cc): host
      shards under their locks, then the SSD log segment by segment; the xbox
      delta_score reset is applied in place in both tiers;
    * shrink applies the accessor rule to both tiers (SSD records rewritten in
      place, deleted ones become tombstones) and compacts the log when under
      half of it is live;
    * point operations (probe / read / insert / assign, used by model loads
      and merges) first promote the keys' SSD rows into the host tier."""

    def __init__(self, host: HostTable, ssd: Optional[SsdTier] = None):
        self.host = host
        self.ssd = ssd
        self.dim = host.dim
        self.stride = host.stride
        self.device = torch.device("cpu")
        self.codec = None  # rows are canonical fp32 in both tiers

    def _ssd_live(self) -> bool:
        return self.ssd is not None and len(self.ssd) > 0

    def promote(self, h: torch.Tensor) -> int:
        """Move the SSD rows of keys h into the host tier; returns how many."""
        if not self._ssd_live():
            return 0
        h = h.reshape(-1).cpu()
        miss = h[self.host.probe(h) < 0]
        if miss.numel() == 0:
            return 0
        found, vals = self.ssd.get(miss)
        if not bool(found.any()):
            return 0
        mk = miss[found]
        rows, _ = self.host._native.insert(mk)
        self.host._native.scatter(rows, vals[found])
        self.ssd.delete(mk)
        return int(mk.numel())

    def probe(self, h: torch.Tensor, n_dev=None) -> torch.Tensor:
        self.promote(h)
        return self.host.probe(h)

    def read(self, h: torch.Tensor) -> torch.Tensor:
        self.promote(h)
        return self.host.read(h)

    def insert_mixed(self, h: torch.Tensor, sgd: SparseSGDConfig, init_embedx: bool = False, n_dev=None) -> int:
        self.promote(h)
        return self.host.insert_mixed(h, sgd, init_embedx)

    def assign(self, h: torch.Tensor, vals: torch.Tensor):
        self.promote(h)
        self.host.assign(h, vals)

    def export(self, with_values: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Every row of both tiers, in memory (small tables and tests; saves
        stream instead)."""
        k, v = self.host.export(with_values)
        if not self._ssd_live():
            return k, v
        sk = self.ssd.keys()
        if not with_values:
            return torch.cat([k, sk]), None
        _, sv = self.ssd.get(sk)
        return torch.cat([k, sk]), torch.cat([v, sv])

    def size(self) -> int:
        return self.host.size() + (len(self.ssd) if self.ssd is not None else 0)

    def shrink(self, cfg: ShrinkConfig) -> int:
        gone = self.host.shrink(cfg)
        if self._ssd_live():
            gone += int(self.ssd._native.shrink(float(cfg.show_click_decay_rate), int(self.host.layout["unseen_days"]),
                                                float(cfg.nonclk_coeff), float(cfg.clk_coeff),
                                                float(cfg.delete_threshold), float(cfg.delete_after_unseen_days)))
            if int(self.ssd._native.live_permille()) < 500:
                self.ssd.compact(0.5)
        return gone

    def save_tiers(self, kind: int, mode: int, reset: bool, cfg, nonclk: float, clk: float, keys_path: str,
                   vals_path: str = "", collect: bool = False):
        """Native streaming save over both tiers: (rows, mixed keys saved or None)."""
        import os

        from .config import SaveConfig

        cfg = cfg or SaveConfig()
        threads = min(16, os.cpu_count() or 4)
        rows, host_rows, ssd_rows, secs, keys = _native.host().save_tiers(
            self.host._native, self.ssd._native if self.ssd is not None else None, int(kind), int(mode), bool(reset),
            float(cfg.base_threshold), float(cfg.delta_threshold), float(cfg.delta_keep_days), float(nonclk),
            float(clk), float(cfg.embedx_threshold), int(self.dim), keys_path, vals_path, threads, bool(collect))
        self.last_save = {"rows": int(rows), "host_rows": int(host_rows), "ssd_rows": int(ssd_rows),
                          "total_s": float(secs), "native": True}
        return int(rows), keys


class TieredStore:
    def __init__(self, engine, host: HostTable, ssd: Optional[SsdTier] = None, sgd: Optional[SparseSGDConfig] = None,
                 spill_unseen: float = 1.0, host_cap_rows: int = 0, retain: bool = True):
        from .gpu_table import GpuSparseTable

        self.engine = engine
        self.host = host
        self.ssd = ssd
        self.sgd = sgd or engine.cfg.sgd
        self.spill_unseen = spill_unseen
        self.host_cap_rows = int(host_cap_rows)
        self.epoch = 0  # pass stamp of host rows: write-back count
        # keep rows the next pass uses again on the GPU across the pass
        # boundary: the staging looks up only keys the live table lacks and
        # the write-back moves only rows the next pass drops
        self.retain = bool(retain)
        self.retained = False  # the last write-back left rows newer than their host copy on the GPU
        live = engine.table
        self.live = live
        if live.codec is not None:
            # codec rows (int16 / SparseAdam / expand / variable) travel in the
            # canonical fp32 layout: export decodes, assign re-encodes, and the
            # host tier's unseen_days column is the canonical one
            c = live.codec
            if host.stride != c.canon_width or host.dim != c.DX:
                raise ValueError(f"tiered store with {c!r}: the host tier must hold canonical rows "
                                 f"(HostTable({c.DX}, stride={c.canon_width}))")
        # staged table: same geometry as the live one
        self.stage_table = GpuSparseTable.like(live)
        self.stream = torch.cuda.Stream(live.device)
        self._stage_thread: Optional[threading.Thread] = None
        self._wb_thread: Optional[threading.Thread] = None
        self._stage_err = None
        self._wb_err = None
        self._wb_lock = threading.Lock()
        # staging (pass n+1) and write-back (pass n) may run at the same time;
        # their host/SSD sections are serialised so a spill cannot pull rows
        # out from under a staging gather
        self._tier_lock = threading.Lock()
        self._staged_keys: Optional[torch.Tensor] = None
        self._staged_src: Optional[torch.Tensor] = None  # the staged pass's keys as given (CPU)
        self._pin = {}  # reusable pinned staging buffers (pinning is slow)
        self.stats = {"stage_s": 0.0, "writeback_s": 0.0, "activate_s": 0.0, "spill_s": 0.0, "ssd_hits": 0,
                      "spilled": 0, "spilled_cap": 0, "staged_rows": 0, "new_rows": 0, "host_rows_staged": 0,
                      "retained_rows": 0, "wb_retained_rows": 0,
                      # phase times of the background threads (seconds, summed)
                      "stage_live_probe_s": 0.0, "stage_wait_s": 0.0, "stage_ssd_get_s": 0.0,
                      "stage_ssd_delete_s": 0.0, "stage_host_s": 0.0, "stage_gpu_s": 0.0, "wb_d2h_s": 0.0,
                      "wb_lock_wait_s": 0.0, "wb_host_insert_s": 0.0, "wb_ssd_delete_s": 0.0,
                      "spill_select_s": 0.0, "spill_put_s": 0.0}

    def _pinned(self, name: str, shape, dtype) -> torch.Tensor:
        n = 1
        for d in shape:
            n *= int(d)
        buf = self._pin.get(name)
        if buf is None or buf.dtype != dtype or buf.numel() < n:
            buf = torch.empty(max(n, 1) * 5 // 4, dtype=dtype, pin_memory=True)
            self._pin[name] = buf
        return buf[:n].view(*shape)

    # ------------------------------------------------------------ staging (FeedPass)
    def stage(self, h: torch.Tensor, block: bool = False):
        """Stage the next pass's (owner-local, unique, mixed) keys into the
        staged GPU table in the background."""
        self.wait_stage()
        self._stage_err = None
        # the write-back in flight now is the one whose host rows this staging
        # must see (a later one waits for THIS staging: joining it would deadlock)
        self._stage_thread = threading.Thread(target=self._stage_run,
                                              args=(h.reshape(-1).cpu().contiguous(), self._wb_thread), daemon=True)
        self._stage_thread.start()
        if block:
            self.wait_stage()

    def _stage_run(self, hc: torch.Tensor, wb_before: Optional[threading.Thread] = None):
        locked = False
        try:
            t0 = time.perf_counter()
            dev = self.live.device
            hd_all = None
            self._staged_src = hc
            if self.retain and self.live.size() > 0:
                # keys the live table already holds come from it at activation
                # (newest values): only the rest is looked up in the host / SSD
                # tiers.  The probe only reads keys -- the running pass updates
                # values, never the key set -- so it runs beside the training.
                with torch.cuda.device(dev), torch.cuda.stream(self.stream):
                    hd_all = hc.to(dev, non_blocking=True)
                    outside = (self.live.probe(hd_all) < 0).cpu()
                hc_all, hc = hc, hc[outside]
                self.stats["retained_rows"] += int(hc_all.numel() - hc.numel())
            tq = time.perf_counter()
            self.stats["stage_live_probe_s"] += tq - t0
            if wb_before is not None:
                wb_before.join()  # host values of earlier passes must be final (its error: wait_writeback)
            self._tier_lock.acquire()
            locked = True
            tl = time.perf_counter()
            self.stats["stage_wait_s"] += tl - tq
            rows = self.host.probe(hc)
            miss = rows < 0
            if self.ssd is not None and bool(miss.any()):
                t_s = time.perf_counter()
                found, vals = self.ssd.get(hc[miss])
                self.stats["stage_ssd_get_s"] += time.perf_counter() - t_s
                if bool(found.any()):
                    mk = hc[miss][found]
                    r, _ = self.host._native.insert(mk)
                    self.host._native.scatter(r, vals[found])
                    self.host._native.stamp(r, self.epoch)  # reloaded for the coming pass: newest
                    t_d = time.perf_counter()
                    self.ssd.delete(mk)
                    self.stats["stage_ssd_delete_s"] += time.perf_counter() - t_d
                    self.stats["ssd_hits"] += int(mk.numel())
                    # the reloaded keys' host rows are known: no second probe
                    # of every staged key
                    at = miss.nonzero().squeeze(1)[found]
                    rows[at] = r.to(rows.dtype)
                    miss[at] = False
            known = ~miss
            kh = hc[known]
            buf = self._pinned("stage", (int(kh.numel()), self.host.stride), torch.float32)
            self.host._native.gather(rows[known].contiguous(), buf)
            self._tier_lock.release()
            locked = False
            tg = time.perf_counter()
            self.stats["stage_host_s"] += tg - tl
            with torch.cuda.device(dev), torch.cuda.stream(self.stream):
                st = self.stage_table
                st.clear()
                hd = hd_all if hd_all is not None else hc.to(dev, non_blocking=True)
                st.insert_mixed(hd, self.sgd)  # new keys get the standard GPU init
                if kh.numel():
                    st.assign(kh.to(dev, non_blocking=True), buf.to(dev, non_blocking=True))
                self._staged_keys = hd
                self.stream.synchronize()
            self.stats["stage_gpu_s"] += time.perf_counter() - tg
            self.stats["staged_rows"] += int(kh.numel())
            self.stats["host_rows_staged"] += int(kh.numel())
            self.stats["new_rows"] += int(miss.sum())
            self.stats["stage_s"] += time.perf_counter() - t0
        except BaseException as e:  # surfaced by wait_stage
            self._stage_err = e
            if locked:
                self._tier_lock.release()

    def restage(self):
        """Stage the already-staged next pass again: its rows were gathered
        before a between-pass mutation of the tiers (ShrinkTable) that they
        must see."""
        self.wait_stage()
        if self._staged_keys is not None and self._staged_src is not None:
            self.stage(self._staged_src)

    def staged_tables(self):
        """The GPU tables whose rows become (or stay) live at the next
        activation: the live table, plus the staged one when a pass is staged."""
        self.wait_stage()
        return [self.live] + ([self.stage_table] if self._staged_keys is not None else [])

    def wait_stage(self):
        if self._stage_thread is not None:
            self._stage_thread.join()
            self._stage_thread = None
        if self._stage_err is not None:
            e, self._stage_err = self._stage_err, None
            raise e

    # ------------------------------------------------------------ BeginPass
    def activate(self):
        """Make the staged pass live: shared keys take the live table's newest
        rows, then the staged table is copied over the live one."""
        self.wait_stage()
        if self._staged_keys is None:
            return
        t0 = time.perf_counter()
        live, st = self.live, self.stage_table
        cur = torch.cuda.current_stream(live.device)
        cur.wait_stream(self.stream)
        k = self._staged_keys
        if live.size() > 0:
            rl = live.probe(k)
            shared = rl >= 0
            if bool(shared.any()):
                st.t.assign(st.probe(k[shared]), live.values[rl[shared]].contiguous())
        live.t.copy_from(st.t)
        self._staged_keys = None
        torch.cuda.synchronize(live.device)
        self.stats["activate_s"] += time.perf_counter() - t0

    # ------------------------------------------------------------ EndPass
    def writeback(self, block: bool = False, full: bool = False):
        """Export the live table and move it into the host tier (then spill
        cold rows to SSD) in the background.  With ``retain`` and the next
        pass staged, rows the next pass uses again stay on the GPU (activation
        carries them over) and only the others are written back -- the
        background thread waits for the staging to know which; ``full``
        (flush: a save / shrink needs the host tier current) writes every row.
        ``retained`` is final once ``wait_writeback`` returns."""
        self.wait_writeback()
        k, v = self.live.export(True)  # device copies: the live table may change after this
        self.retained = False
        filt = self.retain and not full and (self._stage_thread is not None or self._staged_keys is not None)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.live.device))  # the export kernel has to finish first
        self._wb_err = None
        self._wb_thread = threading.Thread(target=self._wb_run, args=(ev, k, v, filt), daemon=True)
        self._wb_thread.start()
        if block:
            self.wait_writeback()

    def _wb_run(self, ev, k, v, filt):
        try:
            t0 = time.perf_counter()
            dev = self.live.device
            with torch.cuda.device(dev), torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                if filt:
                    st = self._stage_thread
                    if st is not None:
                        st.join()  # its error surfaces at the next wait_stage
                    if self._staged_keys is not None and k.numel():
                        keep = self.stage_table.probe(k) < 0  # not in the next pass: evicted from the GPU
                        n_ret = int(k.numel()) - int(keep.sum())
                        if n_ret:
                            k, v = k[keep], v[keep]
                            self.retained = True
                            self.stats["wb_retained_rows"] += n_ret
                kh = self._pinned("wb_keys", tuple(k.shape), k.dtype)
                vh = self._pinned("wb_vals", tuple(v.shape), v.dtype)
                kh.copy_(k, non_blocking=True)
                vh.copy_(v, non_blocking=True)
                self.stream.synchronize()
            del k, v
            tw = time.perf_counter()
            self.stats["wb_d2h_s"] += tw - t0
            with self._tier_lock:
                self.stats["wb_lock_wait_s"] += time.perf_counter() - tw
                self._wb_locked(kh, vh)
            self.stats["writeback_s"] += time.perf_counter() - t0
        except BaseException as e:
            self._wb_err = e

    def _wb_locked(self, kh, vh):
        """Host scatter of the written-back rows, then the SSD spill (holds the tier lock)."""
        self.epoch += 1
        t_i = time.perf_counter()
        rows, fresh = self.host._native.insert_fresh(kh)
        self.host._native.scatter(rows, vh)
        self.host._native.stamp(rows, self.epoch)
        t_d = time.perf_counter()
        self.stats["wb_host_insert_s"] += t_d - t_i
        if self.ssd is not None and len(self.ssd) > 0 and bool(fresh.any()):
            # a key re-entering the host tier may still have a copy on SSD
            # (spilled by an earlier write-back while its pass was live):
            # the host row is newer -- one tier per key
            self.ssd.delete(kh[fresh])
        self.stats["wb_ssd_delete_s"] += time.perf_counter() - t_d
        if self.ssd is not None:
            l = self.host.layout
            t0 = time.perf_counter()
            if self.spill_unseen >= 0:
                ck, cv = self.host._native.select_ge(l["unseen_days"], float(self.spill_unseen))
                if ck.numel():
                    self.ssd.put(ck, cv)
                    self.host.erase(ck)
                    self.stats["spilled"] += int(ck.numel())
            if self.host_cap_rows > 0:
                t_sel = time.perf_counter()
                ck, cv = self.host._native.spill_oldest(self.host_cap_rows)
                t_put = time.perf_counter()
                self.stats["spill_select_s"] += t_put - t_sel
                if ck.numel():
                    self.ssd.put(ck, cv)
                    self.stats["spill_put_s"] += time.perf_counter() - t_put
                    self.stats["spilled"] += int(ck.numel())
                    self.stats["spilled_cap"] += int(ck.numel())
            self.stats["spill_s"] += time.perf_counter() - t0

    def wait_writeback(self):
        with self._wb_lock:
            if self._wb_thread is not None:
                self._wb_thread.join()
                self._wb_thread = None
            if self._wb_err is not None:
                e, self._wb_err = self._wb_err, None
                raise e

    def flush(self):
        """Synchronous write-back of every live row (a save / shrink in the
        middle of a pass, or after an EndPass that retained rows)."""
        self.writeback(block=True, full=True)
