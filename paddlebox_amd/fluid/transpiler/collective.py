"""Collective transpilers (``py/fluid/transpiler/collective.py:37-740``).

The reference rewrites the program: it scales the loss gradient by
1/nranks and inserts ``c_allreduce_sum`` per gradient (GradAllReduce), keeps
parameter snapshots and averages ``snapshot - param`` after each update
(LocalSGD), or all-gathers gradients and runs one Adam per gathered gradient
(MultiThread ``all_gather``) / all-reduces ``coalesce_tensor`` fused segments
(``fuse_all_reduce``).

Here the dense parameters and gradients already live in one contiguous
arena, so a transpiler only records the sync *mode* on the program; the
executor runs it as ONE collective over the arena (parallel/dense.py
``DenseSync.apply``) instead of per-gradient ops.  The ops the reference
would insert are listed in ``program._collective["ops"]`` for inspection.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Union


class Collective:
    mode = "grad_allreduce"

    def __init__(self, nrings: int = 1):
        self.nrings = nrings
        self.nranks = 1
        self.rank = 0
        self.endpoints: List[str] = []
        self.current_endpoint = ""

    def transpile(self, startup_program, main_program, rank: int, endpoints: Union[str, Sequence[str]],
                  current_endpoint: str = "", wait_port: bool = True):
        eps = endpoints.split(",") if isinstance(endpoints, str) else list(endpoints)
        self.endpoints = eps
        self.nranks = len(eps)
        self.rank = int(rank)
        self.current_endpoint = current_endpoint
        self.startup_program = startup_program
        self.main_program = main_program
        main_program._collective = {
            "mode": self._sync_mode(),
            "nranks": self.nranks,
            "rank": self.rank,
            "nrings": self.nrings,
            "k": 1,
            "endpoints": eps,
            "ops": self._ops(),
            "transpiler": type(self).__name__,
        }
        main_program._version += 1
        if startup_program is not None:
            startup_program._collective = {"comm_init": "c_comm_init_all" if self.nranks <= 1 else "c_gen_nccl_id"}

    def _sync_mode(self) -> str:
        return self.mode

    def _ops(self) -> List[str]:
        return ["scale(loss@GRAD, 1/nranks)", "c_allreduce_sum(arena.grad)"]


class GradAllReduce(Collective):
    mode = "grad_allreduce"

    def __init__(self, nrings: int = 2):
        super().__init__(nrings)


class LocalSGD(Collective):
    """Parameter averaging after every local update (snapshot - param is
    all-reduced; ``collective.py:317-418``) == model averaging with k=1."""

    mode = "local_sgd"

    def __init__(self, nrings: int = 2):
        super().__init__(nrings)

    def _ops(self):
        return ["elementwise_sub(snapshot, param)", "c_allreduce_sum", "scale(1/nranks)", "assign(snapshot)"]


class SingleProcessMultiThread(GradAllReduce):
    mode = "grad_allreduce"

    def __init__(self):
        super().__init__(1)


class MultiThread(GradAllReduce):
    """"box" mode: ``all_reduce`` (default), ``fuse_all_reduce`` (the arena
    is already one fused buffer) or ``all_gather`` (gather all gradients, one
    optimizer update per gathered gradient)."""

    def __init__(self, nrings: int = 1, trans_mode: str = "all_reduce"):
        super().__init__(nrings)
        self.trans_mode = trans_mode
        self.fuse_grad_size_in_num = 128
        self.gpu_num = len(os.getenv("FLAGS_selected_gpus", "0").split(","))

    def _sync_mode(self):
        return "allgather" if self.trans_mode == "all_gather" else "grad_allreduce"

    def _ops(self):
        if self.trans_mode == "all_gather":
            return ["c_allgather(arena.grad)", "split", "adam x nranks"]
        if self.trans_mode == "fuse_all_reduce":
            return ["coalesce_tensor (arena)", "c_allreduce_sum"]
        return ["c_allreduce_sum(arena.grad)"]
