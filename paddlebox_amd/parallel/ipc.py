"""In-house IPC mesh collectives for the GPUs of one node
(``csrc/hip/ipc.hip``): peer-to-peer writes over xGMI into IPC-mapped inboxes,
one kernel per collective, no host synchronisation, graph-capturable.

* ``allreduce_(t)`` -- one-shot all-reduce (every rank writes its whole
  buffer into every peer's inbox and sums the W copies: one xGMI hop, for
  latency-bound sizes) or two-phase (reduce-scatter + all-gather: each rank
  moves 2(W-1)/W of the buffer over its 7 links in parallel instead of W-1
  copies; the default above 256 KB).
* ``exchange(send, dst, counts=...)`` -- all-to-all of per-peer record slots
  (the key / value / gradient exchange of the sharded sparse step): only
  ``counts[p]`` records of slot p travel, the receiver copies them into
  ``dst``, gets the counts in ``rcounts`` and, with ``fill_tail``, -1 keys
  past them.  The inbox slot is consumed inside the launch, so nothing the
  caller does between collectives can race a peer's next write.

Reference: the c_mixallgather / heter_comm peer copies
(``c_mixallgather_op.cc:221-327``, ``heter_comm_inl.h:273-490``); here the
memory handles are exchanged once over the process group and every later
call is a single kernel.  Every rank must issue the same sequence of
collectives on a mesh (as with RCCL).  A launch reads the mesh epoch from
device memory, so two collectives of one mesh must never be in flight at once:
a mesh built with ``stream=<name>`` issues every launch on that named side
stream (forked from and joined back into the caller's stream), which orders
them -- the dense mesh uses the dense-sync stream, where the gradient
all-reduce (DenseSync.launch issues there), a data_norm statistics
all-reduce from the tower's dW stream and a transpiled c_allreduce_sum from
the compute stream then queue in issue order.
The sparse exchange meshes are only ever issued from one stream and skip it.  A peer that never arrives makes the
wait time out: the sticky error poisons the results (NaN sums, empty
exchanges) and :meth:`check` raises on the host, instead of hanging the GPU
or training on stale slots.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import _native

# s_sleep(2) polls (~55 ns each) before a wait gives up: ~3.7 s by default, so
# a peer that is seconds late at a pass boundary does not trip it
DEFAULT_SPIN_LIMIT = int(os.environ.get("PBX_IPC_SPIN_LIMIT", str(1 << 26)))


class IpcMeshError(RuntimeError):
    pass


_TRACE = os.environ.get("PBX_IPC_TRACE", "0") == "1"
_VERIFY = os.environ.get("PBX_IPC_VERIFY", "0") == "1"
_N_MESHES = [0]


class IpcMesh:
    def __init__(self, slot_bytes: int, group=None, device=None, blocks: Optional[int] = None, depth: int = 2,
                 spin_limit: Optional[int] = None, stream: Optional[str] = None, self_test: bool = True):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.world > 8:
            raise ValueError("IpcMesh spans the GPUs of one node (<= 8 ranks)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.slot_bytes = (int(slot_bytes) + 15) // 16 * 16
        self.depth = int(depth)
        self.mesh_id = _N_MESHES[0]
        _N_MESHES[0] += 1
        self.calls = 0
        h = _native.hip()
        W = self.world
        if blocks is None:
            # ~16 KB of payload per workgroup (4 x 16 B in flight per lane:
            # about one pass of the unrolled copy loop), so the puts and the
            # copy-out are not latency-bound; 16..64 workgroups -- more cost
            # more in the arrive / publish / wait than they save in the copy
            # (1-rank exchange of a 10 MB slot: 64 blocks 10.3 us, 256 blocks
            # 17.6 us, 16 blocks 17.0 us; profiles/r6_ipc_exchange_bench.txt)
            # (PBX_IPC_MAX_BLOCKS caps it: every workgroup of every rank's
            # collective must be resident at once -- the waits spin -- which
            # matters when several ranks share one GPU, see bench --same-gpu)
            cap = int(os.environ.get("PBX_IPC_MAX_BLOCKS", "64"))
            blocks = max(min(16, cap), min(cap, (W * self.slot_bytes) >> 14))
        # power of two: the arrive / depart counters find the last block by
        # count % grid and wrap at 2^32
        blocks = 1 << max(0, int(blocks).bit_length() - 1)
        # inbox + flags: written by peers over xGMI while this GPU's kernels
        # spin on them, so they live in uncached device memory
        # (hipExtMallocWithFlags, hipDeviceMallocUncached; PBX_IPC_MEM=fine:
        # fine-grained) -- not on the caching allocator, whose coarse-grained
        # hipMalloc memory is only coherent across devices at dispatch / sync
        # boundaries
        self.mem_kind = os.environ.get("PBX_IPC_MEM", "uncached")
        unc = self.mem_kind != "fine"
        dix = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.inbox = h.ipc_buffer(self.depth * 2 * W * self.slot_bytes, dix, unc)
        self.flags = h.ipc_buffer(2 * W * 8, dix, unc).view(torch.int64)
        self.state = torch.zeros(4, dtype=torch.int64, device=self.device)
        self.comm = h.IpcComm(self.rank, W, self.slot_bytes, self.state, int(blocks), self.depth,
                              int(spin_limit or DEFAULT_SPIN_LIMIT))
        # every launch of this mesh in issue order on one named side stream (or the caller's)
        if stream is not None:
            from ..runtime.streams import side_stream

            self.stream = side_stream(self.device, stream)
        else:
            self.stream = None
        self._opened = []
        # no rank may raise between the collectives below (a peer would block
        # in them forever): failures are recorded and agreed on at the end
        err = None
        try:
            mine = (h.ipc_handle(self.inbox), h.ipc_handle(self.flags))
        except Exception as e:  # pragma: no cover - depends on the driver
            mine, err = None, f"export: {e!r}"
        allh = [None] * W
        if W > 1:
            dist.all_gather_object(allh, mine, group=group)
        else:
            allh = [mine]
        for p in range(W):
            if err is not None:
                break
            if p == self.rank:
                self.comm.set_peer(p, self.inbox.data_ptr(), self.flags.data_ptr())
                continue
            if allh[p] is None:
                err = f"rank {p} could not export its inbox"
                break
            try:
                (ih, io), (fh, fo) = allh[p]
                ip = h.ipc_open(ih, io)
                self._opened.append(ip - io)
                fp = h.ipc_open(fh, fo)
                self._opened.append(fp - fo)
                self.comm.set_peer(p, ip, fp)
            except Exception as e:  # pragma: no cover - depends on the driver
                err = f"open peer {p}: {e!r}"
        torch.cuda.synchronize(self.device)
        if W > 1:
            bad = self._all_min(0 if err else 1) == 0
        else:
            bad = err is not None
        if bad:
            self.close()
            raise IpcMeshError(f"IPC mesh setup failed on some rank (this rank: {err or 'ok'})")
        # every construction proves the mesh end to end: known payloads through
        # both exchange phases and both all-reduce forms, checked word by word
        # and agreed on by all ranks (a collective: every rank constructs)
        if self_test:
            # at the default wait bound (construction skew between ranks can
            # exceed a short one), aligned by a barrier
            lim = self.comm.spin_limit()
            self.comm.set_spin_limit(max(lim, DEFAULT_SPIN_LIMIT))
            if W > 1:
                dist.barrier(group=group)
            ok = self.self_test(agree=True)
            self.comm.set_spin_limit(lim)
            if not ok:
                self.close()
                raise IpcMeshError("IPC mesh self-test failed on some rank (payload / count mismatch)")

    def _all_min(self, v: int) -> int:
        t = torch.tensor([int(v)], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            t = t.to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def allreduce_(self, t: torch.Tensor, average: bool = False, two_phase: Optional[bool] = None) -> torch.Tensor:
        """In-place sum (or mean) over the ranks of a contiguous f32 tensor."""
        if two_phase is None:
            two_phase = self.world > 2 and t.numel() * 4 > (256 << 10)
        with self._serial("allreduce"):
            self.comm.allreduce(t, t, 1.0 / self.world if average else 1.0, bool(two_phase))
        return t

    class _Serial:
        def __init__(self, mesh):
            self.m = mesh

        def __enter__(self):
            self.cur = torch.cuda.current_stream(self.m.device)
            self.fork = self.m.stream is not None and self.cur != self.m.stream
            if self.fork:
                self.m.stream.wait_stream(self.cur)
                self.ctx = torch.cuda.stream(self.m.stream)
                self.ctx.__enter__()

        def __exit__(self, *exc):
            if self.fork:
                self.ctx.__exit__(*exc)
                self.cur.wait_stream(self.m.stream)
            return False

    def _serial(self, op: str = ""):
        self.calls += 1
        if _TRACE:
            import sys
            import traceback

            where = " <- ".join(f"{f.name}:{f.lineno}" for f in traceback.extract_stack(limit=6)[:-2][::-1])
            print(f"[ipc r{self.rank} m{self.mesh_id}] {op} #{self.calls} stream={torch.cuda.current_stream(self.device).stream_id} "
                  f"capturing={torch.cuda.is_current_stream_capturing()} {where}", file=sys.stderr, flush=True)
        return IpcMesh._Serial(self)

    def exchange(self, send: torch.Tensor, dst: Optional[torch.Tensor] = None, counts: Optional[torch.Tensor] = None,
                 rec_bytes: int = 16, fill_tail: bool = False, rcounts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """send / dst: [world, slot_bytes] bytes (any dtype, contiguous).  Slot
        p of send goes to peer p (its first counts[p] records of rec_bytes,
        or the whole slot); dst receives slot q from peer q.  Returns dst."""
        if dst is None:
            dst = torch.empty_like(send)
        with self._serial("exchange"):
            self.comm.exchange(send, dst, counts, int(rec_bytes), bool(fill_tail), rcounts)
        return dst

    def pack_exchange(self, uniq_h: torch.Tensor, u_count: torch.Tensor, cap: int, send_index: torch.Tensor,
                      ocnt: torch.Tensor, overflow: torch.Tensor, dst: torch.Tensor,
                      rcounts: torch.Tensor) -> torch.Tensor:
        """The sharded pull's key exchange with the owner pack fused in: the
        unique keys uniq_h[:u_count[0]] go straight to their owners' inbox
        slots (send_index[u] = owner * cap + position, ocnt = per-owner
        counts, zero on entry); dst [world, cap] receives every peer's keys
        (tail -1), rcounts their counts.  One launch instead of pack + send
        buffer + exchange (ipc.hip k_ipc_pack_exchange)."""
        with self._serial("pack_exchange"):
            self.comm.pack_exchange(uniq_h, u_count, int(cap), send_index, ocnt, overflow, dst, rcounts)
        return dst

    def error(self) -> bool:
        """True once any wait on this mesh timed out (device read: syncs)."""
        return bool(int(self.state[2].item()) != 0)

    def check(self):
        """Raise if a collective on this mesh failed (call outside the hot
        loop: at pass ends, checkpoints and the end of a benchmark).  With
        PBX_IPC_VERIFY=1 (debug) every check also re-runs the payload
        self-test -- a collective: every rank checks at the same points."""
        if self.world > 1 and self.error():
            raise IpcMeshError(f"IPC mesh rank {self.rank}: a peer did not arrive within the spin bound; "
                               "results since then are poisoned (NaN / empty)")
        if _VERIFY and self.world > 1 and not torch.cuda.is_current_stream_capturing():
            if not self.self_test(agree=True):
                raise IpcMeshError(f"IPC mesh rank {self.rank}: periodic payload self-test failed")

    def memory_attrs(self):
        """hipPointerGetAttributes (type, device, allocation flags) of the inbox and flags."""
        h = _native.hip()
        return h.ptr_attrs(self.inbox.data_ptr()), h.ptr_attrs(self.flags.data_ptr())

    def self_test(self, agree: bool = True) -> bool:
        """Exchange known patterns with every peer (both phases, several
        slots) and verify them on the host.  agree=True all-reduces the
        verdict over the process group, so every rank takes the same
        fallback decision."""
        W, sb = self.world, self.slot_bytes
        ok = True
        n = min(sb // 8, 4096)
        for it in range(2 * self.depth):
            send = torch.full((W, sb // 8), -7, dtype=torch.int64, device=self.device)
            cnt = torch.empty(W, dtype=torch.int32, device=self.device)
            for p in range(W):
                c = max(1, (n * (p + 1 + it)) // (W + 2 * self.depth))
                cnt[p] = c
                send[p, :c] = (self.rank << 40) + (p << 32) + it * 1000 + torch.arange(c, device=self.device)
            rc = torch.zeros(W, dtype=torch.int32, device=self.device)
            recv = self.exchange(send, None, cnt, 8, True, rc).view(torch.int64).view(W, sb // 8)
            torch.cuda.synchronize(self.device)
            for src in range(W):
                c = max(1, (n * (self.rank + 1 + it)) // (W + 2 * self.depth))
                want = (src << 40) + (self.rank << 32) + it * 1000 + torch.arange(c, device=self.device)
                ok &= int(rc[src]) == c and bool((recv[src, :c] == want).all()) and bool((recv[src, c:] == -1).all())
            na = max(4, min(1000, sb // 4))
            t = torch.arange(na, dtype=torch.float32, device=self.device) + self.rank
            self.allreduce_(t, two_phase=bool(it & 1))
            want = torch.arange(na, dtype=torch.float32, device=self.device) * W + W * (W - 1) / 2
            ok &= bool(torch.allclose(t, want))
        ok &= not self.error()
        if agree and W > 1:
            ok = self._all_min(1 if ok else 0) == 1
        return ok

    def close(self):
        h = _native.hip()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            h.ipc_close(p)
        self._opened = []
