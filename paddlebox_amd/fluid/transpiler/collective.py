"""Collective transpilers (``py/fluid/transpiler/collective.py:37-740``).

They rewrite the program the way the reference does, with ops the executor
runs after backward (``op_role`` = backward) or after the optimizer update
(``op_role`` = optimize), on the ``@GRAD`` / parameter values of the dense
arena:

* ``GradAllReduce``: gradients in segments of ``fuse_grad_size_in_num``, each
  ``coalesce_tensor`` -> ``c_allreduce_sum`` -> ``scale(1/nranks)``
  (``collective.py:258-315``; the reference scales ``loss@GRAD`` instead,
  which is the same update).  Because the dense arena already holds the
  gradients contiguously, a segment's fused buffer IS a slice of the arena
  (``coalesce_tensor`` does not copy), so one segment = one RCCL all-reduce.
* ``LocalSGD``: the startup program snapshots every parameter; after each
  update ``delta = snapshot - param``, ``c_allreduce_sum(delta)``,
  ``scale(1/nranks)``, ``param = snapshot - delta``, ``snapshot = param``
  (``collective.py:317-418``).
* ``MultiThread``: "box" mode -- ``all_reduce`` (as GradAllReduce),
  ``fuse_all_reduce`` (one segment for all gradients), or ``all_gather``:
  ``coalesce_tensor`` -> ``c_allgather`` of the fused gradients and one
  optimizer update per gathered gradient (``collective.py:499-636``).

``program._collective`` keeps the summary (mode, ranks, endpoints) for the
executor and for inspection; the executor's own dense sync is disabled for a
rewritten program because the program now carries it.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Union

OP_ROLE_FORWARD = 0
OP_ROLE_BACKWARD = 1
OP_ROLE_OPTIMIZE = 2


def _params(main_program):
    blk = main_program.global_block()
    if main_program._optimize is not None:
        names = list(main_program._optimize["params"])
        return [blk.var(n) for n in names if blk.has_var(n)]
    return [p for p in blk.all_parameters() if getattr(p, "trainable", True)]


def _grad_var(blk, p):
    name = p.name + "@GRAD"
    if blk.has_var(name):
        return blk.var(name)
    return blk.create_var(name=name, shape=p.shape, dtype=p.dtype, stop_gradient=True)


class Collective:
    mode = "grad_allreduce"

    def __init__(self, nrings: int = 1):
        self.nrings = nrings
        self.nranks = 1
        self.rank = 0
        self.endpoints: List[str] = []
        self.current_endpoint = ""
        self.fuse_grad_size_in_num = 128
        self._seg = 0

    def transpile(self, startup_program, main_program, rank: int, endpoints: Union[str, Sequence[str]],
                  current_endpoint: str = "", wait_port: bool = True):
        eps = endpoints.split(",") if isinstance(endpoints, str) else list(endpoints)
        self.endpoints = eps
        self.nranks = len(eps)
        self.rank = int(rank)
        self.current_endpoint = current_endpoint
        self.startup_program = startup_program
        self.main_program = main_program
        if startup_program is not None:
            self._transpile_startup_program(startup_program, main_program)
        self._transpile_main_program(main_program)
        main_program._collective = {
            "mode": self._sync_mode(),
            "rewritten": True,
            "nranks": self.nranks,
            "rank": self.rank,
            "nrings": self.nrings,
            "k": 1,
            "endpoints": eps,
            "transpiler": type(self).__name__,
        }
        main_program._version += 1

    # -- startup -----------------------------------------------------------
    def _transpile_startup_program(self, startup, main):
        startup._collective = {"comm_init": "c_comm_init_all" if self.nranks <= 1 else "c_gen_nccl_id",
                               "nranks": self.nranks, "rank": self.rank}

    # -- main --------------------------------------------------------------
    def _sync_mode(self) -> str:
        return self.mode

    def _transpile_main_program(self, main):
        self._insert_allreduce_ops(main, self.fuse_grad_size_in_num)

    def _coalesce(self, blk, grads, role):
        fused = blk.create_var(name=f"FusedGrad_{id(self) & 0xffff:x}_{self._seg}", dtype="float32",
                               stop_gradient=True)
        self._seg += 1
        blk.append_op("coalesce_tensor", inputs={"Input": grads}, outputs={"Output": grads, "FusedOutput": fused},
                      attrs={"copy_data": True, "dtype": "float32", "op_role": role})
        return fused

    def _insert_allreduce_ops(self, main, seg_size):
        blk = main.global_block()
        grads = [_grad_var(blk, p) for p in _params(main)]
        seg_size = max(1, int(seg_size))
        for i in range(0, len(grads), seg_size):
            fused = self._coalesce(blk, grads[i:i + seg_size], OP_ROLE_BACKWARD)
            blk.append_op("c_allreduce_sum", inputs={"X": fused}, outputs={"Out": fused},
                          attrs={"ring_id": i // seg_size % max(1, self.nrings), "use_calc_stream": True,
                                 "op_role": OP_ROLE_BACKWARD})
            blk.append_op("scale", inputs={"X": fused}, outputs={"Out": fused},
                          attrs={"scale": 1.0 / max(1, self.nranks), "bias": 0.0, "bias_after_scale": True,
                                 "op_role": OP_ROLE_BACKWARD})


class GradAllReduce(Collective):
    mode = "grad_allreduce"

    def __init__(self, nrings: int = 2):
        super().__init__(nrings)


class LocalSGD(Collective):
    """Parameter averaging after every local update (``collective.py:317-418``)
    == model averaging with k=1."""

    mode = "local_sgd"
    snapshot_suffix = "@SNAPSHOT"

    def __init__(self, nrings: int = 2):
        super().__init__(nrings)

    def _transpile_startup_program(self, startup, main):
        super()._transpile_startup_program(startup, main)
        sblk = startup.global_block()
        for p in _params(main):
            snap = sblk.create_var(name=p.name + self.snapshot_suffix, shape=p.shape, dtype=p.dtype,
                                   persistable=True)
            src = sblk.var(p.name) if sblk.has_var(p.name) else p
            sblk.append_op("assign", inputs={"X": src}, outputs={"Out": snap})

    def _transpile_main_program(self, main):
        blk = main.global_block()
        for p in _params(main):
            snap = blk.create_var(name=p.name + self.snapshot_suffix, shape=p.shape, dtype=p.dtype, persistable=True)
            delta = blk.create_var(name=p.name + "@DELTA", shape=p.shape, dtype=p.dtype, stop_gradient=True)
            role = {"op_role": OP_ROLE_OPTIMIZE}
            blk.append_op("elementwise_sub", inputs={"X": snap, "Y": p}, outputs={"Out": delta}, attrs=role)
            blk.append_op("c_allreduce_sum", inputs={"X": delta}, outputs={"Out": delta},
                          attrs={"ring_id": 0, "use_calc_stream": True, **role})
            blk.append_op("scale", inputs={"X": delta}, outputs={"Out": delta},
                          attrs={"scale": 1.0 / max(1, self.nranks), "bias": 0.0, "bias_after_scale": True, **role})
            blk.append_op("elementwise_sub", inputs={"X": snap, "Y": delta}, outputs={"Out": p}, attrs=role)
            blk.append_op("assign", inputs={"X": p}, outputs={"Out": snap}, attrs=role)


class SingleProcessMultiThread(GradAllReduce):
    mode = "grad_allreduce"

    def __init__(self):
        super().__init__(1)


class MultiThread(GradAllReduce):
    """"box" mode: ``all_reduce`` (default), ``fuse_all_reduce`` (one fused
    segment) or ``all_gather`` (gather all gradients, one optimizer update per
    gathered gradient)."""

    def __init__(self, nrings: int = 1, trans_mode: str = "all_reduce"):
        super().__init__(nrings)
        self.trans_mode = trans_mode
        self.gpu_num = len(os.getenv("FLAGS_selected_gpus", "0").split(","))

    def _sync_mode(self):
        return "allgather" if self.trans_mode == "all_gather" else "grad_allreduce"

    def _transpile_main_program(self, main):
        if self.trans_mode == "all_gather":
            blk = main.global_block()
            grads = [_grad_var(blk, p) for p in _params(main)]
            fused = self._coalesce(blk, grads, OP_ROLE_BACKWARD)
            gathered = blk.create_var(name=fused.name + "@GATHERED", dtype="float32", stop_gradient=True)
            blk.append_op("c_allgather", inputs={"X": fused}, outputs={"Out": gathered},
                          attrs={"ring_id": 0, "nranks": self.nranks, "op_role": OP_ROLE_BACKWARD,
                                 "per_rank_update": True})
            return
        seg = 1 << 30 if self.trans_mode == "fuse_all_reduce" else self.fuse_grad_size_in_num
        self._insert_allreduce_ops(main, seg)
