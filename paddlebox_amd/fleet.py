"""``paddle.distributed.fleet`` subset used by PaddleBox collective training:
``fleet.init``, ``DistributedStrategy`` (``sharding`` / ``sharding_configs``)
and ``fleet.distributed_optimizer`` -- with ``strategy.sharding`` the dense
optimizer is ZeRO-1 sharded (``ThreadShardingOptimizer``,
``sharding_optimizer.py:1867-2053``; implemented by parallel/sharding.py).

One process per GPU: ranks come from ``torch.distributed`` (RCCL on GPUs,
gloo on CPU); ``fleet.init`` creates the default group from the usual
``RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT`` environment when it is present.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist


class DistributedStrategy:
    def __init__(self):
        self.sharding = False
        self.sharding_configs = {"sharding_degree": 0, "use_calc_stream": False}
        self.without_graph_optimization = True
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_num = 128
        self.nccl_comm_num = 1
        self.localsgd = False
        self.localsgd_configs = {"k_steps": 1}
        self.gradient_merge = False
        self.a_sync = False


class _DistOptimizer:
    def __init__(self, opt, strategy: DistributedStrategy, fleet_obj: "Fleet"):
        self.inner_opt = opt
        self.user_defined_strategy = strategy
        self.fleet = fleet_obj

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        out = self.inner_opt.minimize(loss, startup_program, parameter_list, no_grad_set)
        s = self.user_defined_strategy
        if s.sharding:
            mode, k = "sharding", 1
        elif s.localsgd:
            mode, k = "local_sgd", int(s.localsgd_configs.get("k_steps", 1))
        else:
            mode, k = "grad_allreduce", 1
        loss.block.program._collective = {"mode": mode, "k": k, "nranks": self.fleet.worker_num(),
                                          "rank": self.fleet.worker_index(), "strategy": "fleet"}
        return out

    def __getattr__(self, name):
        return getattr(self.inner_opt, name)


class Fleet:
    def __init__(self):
        self._strategy: Optional[DistributedStrategy] = None
        self._is_collective = True

    def init(self, role_maker=None, is_collective: bool = True, strategy: Optional[DistributedStrategy] = None):
        self._is_collective = is_collective
        self._strategy = strategy
        if not dist.is_initialized() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            dist.init_process_group(backend)
        return self

    def worker_index(self) -> int:
        return dist.get_rank() if dist.is_initialized() else 0

    def worker_num(self) -> int:
        return dist.get_world_size() if dist.is_initialized() else 1

    def is_first_worker(self) -> bool:
        return self.worker_index() == 0

    def barrier_worker(self):
        if dist.is_initialized():
            dist.barrier()

    def distributed_optimizer(self, optimizer, strategy: Optional[DistributedStrategy] = None):
        return _DistOptimizer(optimizer, strategy or self._strategy or DistributedStrategy(), self)


fleet = Fleet()
init = fleet.init
distributed_optimizer = fleet.distributed_optimizer
worker_index = fleet.worker_index
worker_num = fleet.worker_num
