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
        """Inner minimize, then the strategy's program rewrite: sharding ->
        ZeRO-1 (the executor runs ShardedFlatAdam); localsgd -> LocalSGD
        transpile; otherwise GradAllReduce with fused gradient segments
        (``fuse_grad_size_in_num``; one segment with ``fuse_all_reduce_ops``)."""
        from .fluid import framework as fw
        from .fluid.transpiler.collective import GradAllReduce, LocalSGD

        out = self.inner_opt.minimize(loss, startup_program, parameter_list, no_grad_set)
        s = self.user_defined_strategy
        main = loss.block.program
        startup = startup_program or fw.default_startup_program()
        n, r = self.fleet.worker_num(), self.fleet.worker_index()
        if s.sharding:
            main._collective = {"mode": "sharding", "k": 1, "nranks": n, "rank": r, "strategy": "fleet"}
            return out
        eps = self.fleet.worker_endpoints()
        if s.localsgd:
            t = LocalSGD()
            k = int(s.localsgd_configs.get("k_steps", 1))
        else:
            t = GradAllReduce(nrings=max(1, int(s.nccl_comm_num)))
            t.fuse_grad_size_in_num = (1 << 30) if s.fuse_all_reduce_ops else int(s.fuse_grad_size_in_num)
            k = 1
        if k > 1:
            # k-step averaging: the executor's model-averaging sync (DenseSync
            # local_sgd, k) -- the transpiled LocalSGD averages every step
            main._collective = {"mode": "local_sgd", "k": k, "nranks": n, "rank": r, "strategy": "fleet"}
            return out
        t.transpile(startup, main, r, eps, eps[r])
        main._collective["strategy"] = "fleet"
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

    def worker_endpoints(self):
        eps = os.environ.get("PADDLE_TRAINER_ENDPOINTS")
        if eps:
            return eps.split(",")
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        return [f"{host}:{6170 + i}" for i in range(self.worker_num())]

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
