"""Dense optimizers and ``BoxPSOptimizer`` (``paddle.fluid.optimizer`` surface).

``minimize`` only records the optimisation spec on the program; the
executor builds the fused flat-arena optimizer (``parallel/dense.py``) the
first time it runs the program.  Sparse parameters are never touched here:
their update is the BoxPS push inside the embedding op's backward.

Reference: ``py/fluid/optimizer.py`` (SGD/Adam/Adagrad/Momentum) and
``BoxPSOptimizer`` ``:7315-7611`` (records ``program._pipeline_opt`` with
trainer ``BoxPSTrainer`` / device worker ``BoxPSWorker``).
"""
from __future__ import annotations

from typing import List, Optional

from .framework import Parameter, Program, Variable, default_main_program


class Optimizer:
    type = "sgd"

    def __init__(self, learning_rate=0.001, regularization=None, grad_clip=None, name=None, **kw):
        self.lr = float(learning_rate)
        self.regularization = regularization
        self.grad_clip = grad_clip
        self.kw = kw

    def _params(self, program: Program, parameter_list, no_grad_set) -> List[Parameter]:
        no_grad = {v if isinstance(v, str) else v.name for v in (no_grad_set or ())}
        if parameter_list is not None:
            names = [p if isinstance(p, str) else p.name for p in parameter_list]
            ps = [program.global_block().var(n) for n in names]
        else:
            ps = program.all_parameters()
        return [p for p in ps if isinstance(p, Parameter) and p.trainable and not getattr(p, "is_summary", False)
                and p.name not in no_grad]

    def minimize(self, loss: Variable, startup_program=None, parameter_list=None, no_grad_set=None):
        program = loss.block.program
        params = self._params(program, parameter_list, no_grad_set)
        program._optimize = {"optimizer": self, "loss": loss.name, "params": [p.name for p in params]}
        program._version += 1
        return [], [(p, None) for p in params]

    def spec(self) -> dict:
        return {"type": self.type, "lr": self.lr, **self.kw}


class SGDOptimizer(Optimizer):
    type = "sgd"


class MomentumOptimizer(Optimizer):
    type = "momentum"

    def __init__(self, learning_rate, momentum, use_nesterov=False, **kw):
        super().__init__(learning_rate, momentum=float(momentum), use_nesterov=use_nesterov, **kw)


class AdagradOptimizer(Optimizer):
    type = "adagrad"

    def __init__(self, learning_rate, epsilon=1e-6, initial_accumulator_value=0.0, **kw):
        super().__init__(learning_rate, epsilon=float(epsilon),
                         initial_accumulator_value=float(initial_accumulator_value), **kw)


class AdamOptimizer(Optimizer):
    type = "adam"

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, lazy_mode=False, **kw):
        super().__init__(learning_rate, beta1=float(beta1), beta2=float(beta2), epsilon=float(epsilon), **kw)


class AdamWOptimizer(AdamOptimizer):
    type = "adamw"

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, weight_decay=0.01, **kw):
        super().__init__(learning_rate, beta1, beta2, epsilon, weight_decay=float(weight_decay), **kw)


SGD = SGDOptimizer
Momentum = MomentumOptimizer
Adagrad = AdagradOptimizer
Adam = AdamOptimizer
AdamW = AdamWOptimizer


class BoxPSOptimizer:
    """Wraps a dense optimizer and marks the program for the BoxPS trainer.

    ``cut_list``/``place_list`` program sectioning is accepted for API
    compatibility; like the reference worker (``py/fluid/device_worker.py:649-652``
    uses only ``section_program_list[0]``), the whole program runs as one
    section per GPU process."""

    def __init__(self, optimizer: Optimizer, cut_list=None, place_list=None, concurrency_list=None,
                 queue_size=30, sync_steps=1, start_cpu_core_id=0):
        self._optimizer = optimizer
        self._cut_list = cut_list or []
        self._place_list = place_list or []
        self._concurrency_list = concurrency_list or []
        self._sync_steps = sync_steps
        self._start_cpu_core_id = start_cpu_core_id

    def minimize(self, loss: Variable, startup_program=None, parameter_list=None, no_grad_set=None):
        ops, pg = self._optimizer.minimize(loss, startup_program, parameter_list, no_grad_set)
        program = loss.block.program
        need_sync = [p.name for p, _ in pg]
        program._pipeline_opt = {
            "trainer": "BoxPSTrainer",
            "device_worker": "BoxPSWorker",
            "section_program_list": [{"program": program, "input_set": set(), "output_set": set()}],
            "place_list": self._place_list,
            "param_need_sync": need_sync,
            "sync_steps": self._sync_steps,
        }
        return ops, pg
