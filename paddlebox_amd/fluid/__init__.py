"""``paddle.fluid``-compatible static-graph front end for the MI355X engine.

PaddleBox training scripts build a Program with ``fluid.layers`` /
``fluid.contrib.layers``, wrap the optimizer in ``BoxPSOptimizer`` and drive
passes with ``fluid.core.BoxPS`` + ``DatasetFactory`` +
``Executor.train_from_dataset``.  The same script runs here (``import
paddlebox_amd.fluid as fluid``, or ``import paddle.fluid as fluid`` via the
``paddle`` alias package at the repo root); programs are lowered to the
fused gfx950 kernels (see ``lowering.py``).
"""
from . import contrib, core, initializer, io, layers, optimizer, transpiler  # noqa: F401
from .dataset import DatasetFactory  # noqa: F401
from .transpiler import DistributeTranspiler, DistributeTranspilerConfig  # noqa: F401
from .executor import CompiledProgram, Executor  # noqa: F401
from . import collective_kernels  # noqa: F401,E402  (registers the c_* op kernels)
from .framework import (CPUPlace, CUDAPinnedPlace, CUDAPlace, LoDTensor, Parameter, ParamAttr,  # noqa: F401
                        Program, Scope, Variable, WeightNormParamAttr, cpu_places, create_lod_tensor, cuda_places,
                        default_main_program, default_startup_program, global_scope, in_dygraph_mode,
                        is_compiled_with_cuda, name_scope, program_guard, scope_guard, unique_name)
from .optimizer import BoxPSOptimizer  # noqa: F401

DataFeedDesc = None  # protobuf feed descs are replaced by DatasetBase setters
