"""HIP-graph capture of a whole training step.

CTR steps are launch-bound (~100 small kernels: dedup, probe, fused
pull/seqpool, FM, data_norm, MLP GEMMs, loss, push-merge, Adagrad, RCCL
all-reduce, Adam).  Everything in the engine is shape-static and free of host
synchronisation, so the forward, backward, sparse push, dense sync and
optimizer are captured once into a HIP graph and replayed per batch (the
reference instead runs an op list with several stream syncs per batch,
``boxps_worker.cc:1296-1324``).

Input buffers are double-buffered with one graph per buffer set, so the copy
of batch i+1 (copy stream) overlaps the replay of batch i.  The bench and the
device-pass trainer keep whole passes resident in HBM, so that copy is a D2D
gather into the graph's input buffers; host batches (``--inputs host``, the
host-assembly fallback) arrive through one pinned H2D copy per buffer set.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Callable, List, Optional, Sequence

import torch

from .streams import side_stream

from .. import _native
from ..parallel.dense import join_grad_producers


def _tensor_fields(b) -> List[str]:
    return [f.name for f in dataclasses.fields(b) if isinstance(getattr(b, f.name), torch.Tensor)]


def _layout(b):
    lay, off = [], 0
    for f in _tensor_fields(b):
        t = getattr(b, f)
        n = t.numel() * t.element_size()
        lay.append((f, off, n))
        off += (n + 255) // 256 * 256
    return lay, off


def pack_batch(b, device=None, pin: bool = False):
    """Copy a batch's tensors into ONE contiguous byte buffer (256-B aligned
    fields) and return the batch with its tensors as views of it (``_flat``
    holds the buffer), so a whole batch moves host->device in a single copy
    instead of one per field."""
    lay, total = _layout(b)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    flat = torch.empty(total, dtype=torch.uint8, device=dev, pin_memory=pin and dev.type == "cpu")
    kw = {f.name: getattr(b, f.name) for f in dataclasses.fields(b)}
    for f, off, n in lay:
        t = getattr(b, f)
        v = flat[off:off + n].view(t.dtype).view(t.shape)
        v.copy_(t)
        kw[f] = v
    nb = type(b)(**kw)
    nb._flat = flat
    return nb


def clone_batch(b, device):
    return pack_batch(b, device)


def _drain_collective_watchdog(settle_s: float = 0.3):
    """Let the RCCL process group retire the eager collectives of the warm-up
    before a capture starts: synchronize, then give its watchdog thread (100 ms
    poll) time to drop the completed work, so it has no event left to query
    while the capture runs."""
    import time

    import torch.distributed as dist

    torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized():
        time.sleep(settle_s)


class GraphedTrainStep:
    def __init__(self, step_fn: Callable[[Any], Any], example_batch, device, n_buffers: int = 2,
                 warmup: int = 3, max_inflight: int = 3, warm_batches: Sequence[Any] = (),
                 on_warm: Optional[Callable[[Any], None]] = None, prefetch=None, steps_per_graph: int = 1,
                 pipeline=None, join_each_step: bool = True):
        """``steps_per_graph`` K > 1: each graph holds K consecutive training
        steps over K batch buffers (``load`` then takes K host batches and
        ``run`` trains all K).  Inside one graph consecutive steps are
        separated by a kernel boundary only; between graphs the replay pays
        the graph-launch boundary and the wait on the batch copy once per K
        steps.  The constructor's default stays K = 1 (a single-step graph
        is what eager-equivalence tests and the host-input path use); the
        bench and the fluid trainer pass K = 4 with the pipelined front
        (``bench.py --graph-steps``, FLAGS_padbox_train_steps_per_graph),
        where K = 4 vs 2 vs 1 measured 0.362-0.364 vs ~0.368 vs 0.393
        ms/step (profiles/r4_input_stall.txt, r4_graph_steps_ab.txt; the
        round-3 measurement without the pipelined front showed no gain).
        ``prefetch``: optional (engine, keys_of) -- pipelined sparse pull:
        graph j also runs the dedup + probe of buffer j+1's keys on a side
        stream while batch j trains (SparseEngine.prefetch, pull slot = buffer
        index), so each step's pull starts at the seqpool."""
        """``pipeline``: optional (prep, set_next[, clear]) -- pipelined pull with the
        whole front: graph j pools buffer j+1 (dedup + seqpool) at the end of
        its own step, after the sparse push, under the dW GEMM
        (CtrTrainStep.set_next / prefetch); ``prep(buf, j)`` pools buffer j
        eagerly when its graph finds it unprepared, ``set_next(buf, j)`` tells
        the step what to pool (None: nothing), ``clear()`` drops the engine's
        host-side prepared entries.  Load buffers two graphs ahead: graph j
        waits for buffer set j+1's copy.  With K steps per graph, step k
        pools step k+1's batch inside the graph and the last step pools the
        next graph's first (pull slot = batch buffer index: n_buffers * K).
        ``warmup`` eager runs of ``step_fn`` on the example batch precede
        the capture (lazy allocations, kernel selection).  A trainer that must
        not train a batch twice passes ``warmup=0`` and ``warm_batches``: real
        batches run eagerly through the same buffers before the capture
        (``on_warm(out)`` sees each step's outputs)."""
        self.device = torch.device(device)
        self.step_fn = step_fn
        self.fields = _tensor_fields(example_batch)
        self.K = max(1, int(steps_per_graph))
        if self.K > 1 and prefetch is not None:
            raise ValueError("steps_per_graph > 1 does not combine with the pipelined pull")
        if prefetch is not None and pipeline is not None:
            raise ValueError("prefetch and pipeline are alternatives")
        self.pipeline = pipeline
        self.bufs = [clone_batch(example_batch, self.device) for _ in range(n_buffers * self.K)]
        cur = torch.cuda.current_stream(self.device)
        s = side_stream(self.device, "graph_warmup")
        s.wait_stream(cur)
        if pipeline is not None:
            pipeline[1](None, 0)  # eager warm-up steps pool nothing ahead
        with torch.cuda.stream(s):
            for _ in range(warmup):
                step_fn(self.bufs[0])
                join_grad_producers()
            for hb in warm_batches:
                self.bufs[0]._flat.copy_(hb._flat, non_blocking=True)
                out = step_fn(self.bufs[0])
                join_grad_producers()
                if on_warm is not None:
                    on_warm(out)
        cur.wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.prefetch = prefetch
        self._side = side_stream(self.device, "graph_prefetch") if prefetch is not None else None
        # buffer contents versions (bumped by load / fill) and the version each
        # buffer had when a replay prefetched it: a buffer reloaded after its
        # prefetch is prepared again before its own replay
        self._ver = [0] * n_buffers
        self._pref_ver = [-1] * n_buffers
        if prefetch is not None:
            eng, keys_of = prefetch
            eng.clear_prefetch()
            eng.prefetch(keys_of(self.bufs[0]), 0)  # graph 0's pull finds buffer 0 prepared
        if pipeline is not None:
            pipeline[0](self.bufs[0], 0)  # graph 0's pull finds buffer 0 pooled
        nK = n_buffers * self.K  # batch buffers (= pull slots of the pipeline)
        self.graphs = []
        _drain_collective_watchdog()
        # no cyclic garbage collection inside a capture: an unreachable object
        # cycle of an earlier session (tower <-> its hooks) can hold graph
        # execs, events and tensors whose destructors must not run while this
        # thread captures (seen as an abort in a capture right after another
        # session's pass)
        import gc

        gc.collect()
        gc_was = gc.isenabled()
        gc.disable()
        try:
            self._capture_all(n_buffers, nK, prefetch, pipeline, join_each_step, step_fn)
        finally:
            if gc_was:
                gc.enable()
        if prefetch is not None:
            prefetch[0].clear_prefetch()
        if pipeline is not None:
            pipeline[1](None, 0)
            if len(pipeline) > 2:
                pipeline[2]()  # the host-side prepared entries only steer captures
        torch.cuda.synchronize(self.device)
        self.copy_stream = side_stream(self.device, "graph_copy")
        self.ready = [torch.cuda.Event() for _ in range(n_buffers)]
        self.free = [torch.cuda.Event() for _ in range(n_buffers)]
        for e in self.free:
            e.record(cur)
        # Host throttle: replay i waits (on the host) for replay i - max_inflight
        # to finish.  Unthrottled, the host runs tens of steps ahead and the
        # runtime periodically blocks it for 6-12 ms to recycle its launch
        # resources (profiles/r2_h2d_stall.txt) -- far longer than the queued
        # GPU work -- so a bounded queue is both steadier and faster.
        self.max_inflight = max(1, int(max_inflight))
        self.done = [torch.cuda.Event() for _ in range(self.max_inflight)]
        self.step_no = 0

    def _capture_all(self, n_buffers, nK, prefetch, pipeline, join_each_step, step_fn):
        pool = None
        n = n_buffers
        for j in range(n_buffers):
            g = torch.cuda.CUDAGraph()
            # thread_local: RCCL's watchdog thread keeps querying the events of
            # the eager (warm-up) collectives; under the default global mode
            # such a query from another thread invalidates the capture and
            # kills the watchdog (hipErrorStreamCaptureUnsupported)
            with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                if prefetch is not None:
                    eng, keys_of = prefetch
                    cap = torch.cuda.current_stream(self.device)
                    self._side.wait_stream(cap)
                    with torch.cuda.stream(self._side):
                        eng.prefetch(keys_of(self.bufs[(j + 1) % n]), (j + 1) % n)
                for k in range(self.K):
                    if pipeline is not None:
                        # step b pools buffer b+1 after its push (across graphs: the next graph's first)
                        b1 = (j * self.K + k + 1) % nK
                        pipeline[1](self.bufs[b1], b1)
                    out = step_fn(self.bufs[j * self.K + k])
                    if join_each_step or k == self.K - 1:
                        # side streams forked in the step rejoin (before the capture
                        # ends; join_each_step=False: a step's side work may run on
                        # under the next step of the same graph, which joins it)
                        join_grad_producers()
                if prefetch is not None:
                    torch.cuda.current_stream(self.device).wait_stream(self._side)
            pool = g.pool()
            self.graphs.append((g, out))

    @property
    def n(self) -> int:
        """Number of graphs (buffer sets of K batches each)."""
        return len(self.graphs)

    _dev_inputs = None  # host flat data_ptr -> HBM copy (stage_inputs)

    def stage_inputs(self, host_batches):
        """Keep a copy of every (packed) host batch in HBM: load() then moves
        a batch into the graph's input buffers with a device-to-device copy
        instead of a host-to-device DMA.  The per-step input copy stays in
        the step (same bytes, same stream order); what goes away is the HIP
        runtime's host-side block in hipMemcpyAsync from pinned memory, which
        on MI355X stalls the launching thread for 7-19 ms once in the first
        few dozen copies after a synchronisation (bench --trace-timed)."""
        cache = {}
        with torch.cuda.stream(self.copy_stream):
            for hb in host_batches:
                f = getattr(hb, "_flat", None)
                if f is None or f.data_ptr() in cache:
                    continue
                cache[f.data_ptr()] = f.to(self.device, non_blocking=True)
        torch.cuda.synchronize(self.device)
        self._dev_inputs = cache

    def load(self, i: int, host_batch):
        """Async H2D of a (pinned) host batch -- K of them (a sequence) when
        steps_per_graph = K > 1 -- into buffer set i."""
        batches = list(host_batch) if self.K > 1 else [host_batch]
        if len(batches) != self.K:
            raise ValueError(f"load needs {self.K} host batches per buffer set")
        self._ver[i] += 1
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(self.free[i])
            for k, hb in enumerate(batches):
                dst = self.bufs[i * self.K + k]
                src_flat = getattr(hb, "_flat", None)
                dev = self._dev_inputs.get(src_flat.data_ptr()) if (self._dev_inputs and src_flat is not None) else None
                if dev is not None and dev.numel() == dst._flat.numel():
                    dst._flat.copy_(dev, non_blocking=True)  # HBM-resident batch: device-to-device
                elif src_flat is not None and src_flat.numel() == dst._flat.numel():
                    if src_flat.is_pinned():
                        # one raw DMA; reuse of both buffers is ordered by free/ready
                        _native.hip().memcpy_h2d(dst._flat, src_flat)
                    else:
                        dst._flat.copy_(src_flat, non_blocking=True)
                else:
                    for f in self.fields:
                        getattr(dst, f).copy_(getattr(hb, f), non_blocking=True)
            self.ready[i].record(self.copy_stream)

    def invalidate_prefetch(self):
        """Work outside the graphs changed the table (eager steps): every
        buffer set is pooled / prepared again before its next replay."""
        self._pref_ver = [-1] * len(self._pref_ver)

    def fill(self, i: int, fn, stream=None):
        """Produce buffer set i on the device: ``fn(buf)`` enqueues kernels
        that write it (on ``stream``, default the copy stream) once the
        replay that last read it has finished.  With K steps per graph
        ``fn`` is a sequence of K such callables, one per batch buffer."""
        fns = list(fn) if self.K > 1 else [fn]
        if len(fns) != self.K:
            raise ValueError(f"fill needs {self.K} producers per buffer set")
        st = stream if stream is not None else self.copy_stream
        self._ver[i] += 1
        st.wait_event(self.free[i])
        with torch.cuda.stream(st):
            for k, f in enumerate(fns):
                f(self.bufs[i * self.K + k])
        self.ready[i].record(st)

    trace = None  # diagnostics: a list to collect (throttle wait, rest of run) host seconds per replay

    def drained(self):
        """The caller synchronised the device: every replay has finished, so
        the next max_inflight replays need no host-side throttle wait."""
        self.step_no = 0

    def run(self, i: int):
        import time as _t

        t0 = _t.perf_counter() if self.trace is not None else 0.0
        cur = torch.cuda.current_stream(self.device)
        slot = self.step_no % self.max_inflight
        if self.step_no >= self.max_inflight:
            self.done[slot].synchronize()
        t1 = _t.perf_counter() if self.trace is not None else 0.0
        cur.wait_event(self.ready[i])
        if self.pipeline is not None:
            n = len(self.graphs)
            cur.wait_event(self.ready[(i + 1) % n])  # graph i pools buffer set i+1's first batch
            if self._pref_ver[i] != self._ver[i]:
                # buffer set i's first batch was not pooled by the previous
                # replay with its current contents: pool it now
                self.pipeline[0](self.bufs[i * self.K], i * self.K)
                self.pipeline[2]() if len(self.pipeline) > 2 else None
                join_grad_producers()  # side-stream parts of that pooling (PBX_TD_FINISH_SIDE)
            self._pref_ver[(i + 1) % n] = self._ver[(i + 1) % n]
        if self.prefetch is not None:
            n = len(self.bufs)
            cur.wait_event(self.ready[(i + 1) % n])  # graph i prefetches buffer i+1
            if self._pref_ver[i] != self._ver[i]:
                # buffer i was not prefetched with its current contents (first
                # replay, out-of-order use, reloaded after the prefetch):
                # prepare it now, into slot i
                eng, keys_of = self.prefetch
                eng.prefetch(keys_of(self.bufs[i]), i)
                eng.clear_prefetch()
            self._pref_ver[(i + 1) % n] = self._ver[(i + 1) % n]
        g, out = self.graphs[i]
        g.replay()
        self.free[i].record(cur)
        self.done[slot].record(cur)
        self.step_no += 1
        if self.trace is not None:
            self.trace.append((t1 - t0, _t.perf_counter() - t1))
        return out

    def warm(self, host_batches: Sequence[Any], replays: int = 32):
        """Replay the pipelined load+run cycle until it is in steady state.

        Measured on MI355X (profiles/r2_host_diag.txt): the first ~25 replays
        after capture enqueue at ~0.4 ms/step on the host while steady-state
        replays take ~0.03 ms, so a training loop that starts timing right
        after capture would otherwise see the runtime's warm-up, not the step.
        These are ordinary training steps on the given batches."""
        nb = len(host_batches)

        def group(g):
            if self.K == 1:
                return host_batches[g % nb]
            return [host_batches[(g * self.K + k) % nb] for k in range(self.K)]

        self.load(0, group(0))
        for i in range(replays):  # graph launches: the runtime warm-up is per launch
            self.load((i + 1) % self.n, group(i + 1))
            self.run(i % self.n)
        torch.cuda.synchronize(self.device)
