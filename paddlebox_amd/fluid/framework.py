"""Minimal static-graph IR with the ``paddle.fluid`` surface PaddleBox scripts use.

A :class:`Program` is a list of :class:`Operator` records over named
:class:`Variable` s, built by the ``fluid.layers`` functions exactly like the
reference's ProgramDesc/BlockDesc/OpDesc (``paddle/fluid/framework/``,
python side ``py/fluid/framework.py``).  Nothing executes while building: the
:class:`~paddlebox_amd.fluid.executor.Executor` lowers the op list once per
program to a sequence of PyTorch-ROCm / hand-written HIP calls (with
PaddleBox-specific fusions, see ``lowering.py``) and runs it; autograd
provides the backward, so no grad-op makers exist.

Only one block per program is supported (PaddleBox CTR programs have no
control flow).
"""
from __future__ import annotations

import contextlib
import copy
import itertools
from collections import OrderedDict
from typing import Any, Dict, Iterable, List, Optional, Sequence, Union

import numpy as np
import torch

# ----------------------------------------------------------------- unique names
_name_counters: Dict[str, itertools.count] = {}
_name_prefix: List[str] = []


class unique_name:  # noqa: N801  (paddle.fluid.unique_name module surface)
    @staticmethod
    def generate(key: str) -> str:
        c = _name_counters.setdefault(key, itertools.count())
        return f"{key}_{next(c)}"

    @staticmethod
    @contextlib.contextmanager
    def guard(new_generator=None):
        global _name_counters
        saved = _name_counters
        _name_counters = {}
        try:
            yield
        finally:
            _name_counters = saved


@contextlib.contextmanager
def name_scope(prefix: Optional[str] = None):
    _name_prefix.append(prefix or "")
    try:
        yield
    finally:
        _name_prefix.pop()


# ----------------------------------------------------------------- places
class CPUPlace:
    def __repr__(self):
        return "CPUPlace()"

    def device(self) -> torch.device:
        return torch.device("cpu")


class CUDAPlace:
    """A GPU (HIP device) ordinal -- name kept for script compatibility."""

    def __init__(self, dev_id: int = 0):
        self.dev_id = int(dev_id)

    def __repr__(self):
        return f"CUDAPlace({self.dev_id})"

    def get_device_id(self) -> int:
        return self.dev_id

    def device(self) -> torch.device:
        return torch.device("cuda", self.dev_id)


class CUDAPinnedPlace(CPUPlace):
    pass


def cuda_places(device_ids=None):
    n = torch.cuda.device_count()
    ids = range(n) if device_ids is None else device_ids
    return [CUDAPlace(i) for i in ids]


def cpu_places(device_count=1):
    return [CPUPlace() for _ in range(device_count)]


def is_compiled_with_cuda() -> bool:
    return torch.cuda.is_available()


def to_device(place) -> torch.device:
    if place is None:
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if isinstance(place, torch.device):
        return place
    return place.device()


# ----------------------------------------------------------------- variables
_DTYPES = {
    "float32": torch.float32, "float": torch.float32, "fp32": torch.float32,
    "float64": torch.float64, "double": torch.float64,
    "float16": torch.float16, "bfloat16": torch.bfloat16,
    "int64": torch.int64, "uint64": torch.int64, "int32": torch.int32, "int8": torch.int8,
    "bool": torch.bool,
}


def torch_dtype(dtype) -> torch.dtype:
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(dtype, np.dtype) or (isinstance(dtype, type) and issubclass(dtype, np.generic)):
        dtype = np.dtype(dtype).name
    return _DTYPES[str(dtype)]


def dtype_name(dtype) -> str:
    if isinstance(dtype, str):
        return "int64" if dtype == "uint64" else dtype
    return {v: k for k, v in reversed(list(_DTYPES.items()))}[torch_dtype(dtype)]


class Variable:
    """A named value in a block.  ``shape`` uses -1 for the batch dimension."""

    def __init__(self, block: "Block", name: str, shape: Sequence[int] = (), dtype="float32", lod_level: int = 0,
                 persistable: bool = False, stop_gradient: bool = False, is_data: bool = False,
                 type: str = "lod_tensor"):  # noqa: A002
        self.block = block
        self.name = name
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype_name(dtype)
        self.lod_level = int(lod_level)
        self.persistable = persistable
        self.stop_gradient = stop_gradient
        self.is_data = is_data
        self.type = type
        self.op: Optional["Operator"] = None  # producer

    # ---- paddle Variable surface
    @property
    def program(self) -> "Program":
        return self.block.program

    def __repr__(self):
        return f"Var({self.name}, shape={self.shape}, dtype={self.dtype}, lod={self.lod_level})"

    def __str__(self):
        return self.__repr__()

    def to_string(self, throw_on_error=False, with_details=False) -> str:
        return repr(self)

    def astype(self, dtype):
        from .layers import nn as L

        return L.cast(self, dtype)

    # ---- arithmetic -> elementwise ops
    def _binary(self, other, op_type, reverse=False):
        from .layers import nn as L

        if not isinstance(other, Variable):
            if op_type == "elementwise_add":
                return L.scale(self, 1.0, float(other))
            if op_type == "elementwise_sub":
                return L.scale(self, -1.0 if reverse else 1.0, float(other) if reverse else -float(other))
            if op_type == "elementwise_mul":
                return L.scale(self, float(other), 0.0)
            if op_type == "elementwise_div" and not reverse:
                return L.scale(self, 1.0 / float(other), 0.0)
            other = L.fill_constant(shape=[1], dtype=self.dtype, value=float(other))
        x, y = (other, self) if reverse else (self, other)
        return L._elementwise(op_type, x, y)

    def __add__(self, o):
        return self._binary(o, "elementwise_add")

    __radd__ = __add__

    def __sub__(self, o):
        return self._binary(o, "elementwise_sub")

    def __rsub__(self, o):
        return self._binary(o, "elementwise_sub", reverse=True)

    def __mul__(self, o):
        return self._binary(o, "elementwise_mul")

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self._binary(o, "elementwise_div")

    def __rtruediv__(self, o):
        return self._binary(o, "elementwise_div", reverse=True)

    def __neg__(self):
        from .layers import nn as L

        return L.scale(self, -1.0, 0.0)


class Parameter(Variable):
    def __init__(self, block, name, shape, dtype="float32", initializer=None, trainable=True, learning_rate=1.0,
                 regularizer=None, need_clip=True, do_model_average=None, **kw):
        super().__init__(block, name, shape, dtype, persistable=True, stop_gradient=not trainable, **kw)
        self.initializer = initializer
        self.trainable = trainable
        self.optimize_attr = {"learning_rate": float(learning_rate)}
        self.regularizer = regularizer
        self.need_clip = need_clip
        self.do_model_average = do_model_average

    def __repr__(self):
        return f"Param({self.name}, shape={self.shape}, trainable={self.trainable})"


class ParamAttr:
    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None, trainable=True,
                 do_model_average=True, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.do_model_average = do_model_average
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg) -> Optional["ParamAttr"]:
        if arg is None:
            return ParamAttr()
        if arg is False:
            return None
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        # an initializer
        return ParamAttr(initializer=arg)


WeightNormParamAttr = ParamAttr


# ----------------------------------------------------------------- operators
class Operator:
    def __init__(self, block: "Block", type: str, inputs: Dict[str, List[Variable]],  # noqa: A002
                 outputs: Dict[str, List[Variable]], attrs: Dict[str, Any]):
        self.block = block
        self.type = type
        self.inputs = {k: list(v) for k, v in inputs.items()}
        self.outputs = {k: list(v) for k, v in outputs.items()}
        self.attrs = dict(attrs)
        for vs in self.outputs.values():
            for v in vs:
                v.op = self

    def input(self, slot: str) -> List[str]:
        return [v.name for v in self.inputs.get(slot, [])]

    def output(self, slot: str) -> List[str]:
        return [v.name for v in self.outputs.get(slot, [])]

    @property
    def input_arg_names(self) -> List[str]:
        return [v.name for vs in self.inputs.values() for v in vs]

    @property
    def output_arg_names(self) -> List[str]:
        return [v.name for vs in self.outputs.values() for v in vs]

    def attr(self, name: str):
        return self.attrs.get(name)

    def has_attr(self, name: str) -> bool:
        return name in self.attrs

    def _set_attr(self, name, val):
        self.attrs[name] = val

    def __repr__(self):
        ins = {k: [v.name for v in vs] for k, vs in self.inputs.items()}
        outs = {k: [v.name for v in vs] for k, vs in self.outputs.items()}
        return f"{self.type}({ins}) -> {outs}"


# ----------------------------------------------------------------- blocks / programs
class Block:
    def __init__(self, program: "Program", idx: int = 0):
        self.program = program
        self.idx = idx
        self.vars: "OrderedDict[str, Variable]" = OrderedDict()
        self.ops: List[Operator] = []

    def create_var(self, name: Optional[str] = None, shape=(), dtype="float32", lod_level=0, persistable=False,
                   stop_gradient=False, is_data=False, type="lod_tensor", **_) -> Variable:  # noqa: A002
        name = name or unique_name.generate("tmp")
        v = Variable(self, name, shape, dtype, lod_level, persistable, stop_gradient, is_data, type)
        self.vars[name] = v
        self.program._version += 1
        return v

    def create_parameter(self, name, shape, dtype="float32", initializer=None, trainable=True, learning_rate=1.0,
                         **kw) -> Parameter:
        if name in self.vars and isinstance(self.vars[name], Parameter):
            return self.vars[name]  # shared parameter (same ParamAttr name)
        p = Parameter(self, name, shape, dtype, initializer, trainable, learning_rate, **kw)
        self.vars[name] = p
        self.program._version += 1
        return p

    def var(self, name: str) -> Variable:
        if name not in self.vars:
            raise ValueError(f"var {name} not in this block")
        return self.vars[name]

    def has_var(self, name: str) -> bool:
        return name in self.vars

    def append_op(self, type: str, inputs=None, outputs=None, attrs=None) -> Operator:  # noqa: A002
        norm = lambda d: {k: (v if isinstance(v, (list, tuple)) else [v]) for k, v in (d or {}).items()  # noqa: E731
                          if v is not None}
        op = Operator(self, type, norm(inputs), norm(outputs), attrs or {})
        self.ops.append(op)
        self.program._version += 1
        return op

    def all_parameters(self) -> List[Parameter]:
        return [v for v in self.vars.values() if isinstance(v, Parameter)]

    def iter_parameters(self):
        return iter(self.all_parameters())


class Program:
    def __init__(self):
        self.blocks = [Block(self, 0)]
        self.random_seed = 0
        self._version = 0
        self._pipeline_opt: Optional[dict] = None
        self._optimize: Optional[dict] = None  # set by Optimizer.minimize
        self._collective: Optional[dict] = None  # set by transpiler / fleet (dense sync mode)
        self._fleet_opt: Optional[dict] = None
        self._is_test = False
        self._startup: Optional["Program"] = None

    def global_block(self) -> Block:
        return self.blocks[0]

    def block(self, i: int) -> Block:
        return self.blocks[i]

    def current_block(self) -> Block:
        return self.blocks[0]

    @property
    def num_blocks(self) -> int:
        return len(self.blocks)

    def list_vars(self) -> Iterable[Variable]:
        return iter(self.global_block().vars.values())

    def all_parameters(self) -> List[Parameter]:
        return self.global_block().all_parameters()

    def clone(self, for_test: bool = False) -> "Program":
        """Copy of the op list; ``for_test`` drops the optimizer so the
        executor runs forward only (and data_norm stops updating)."""
        p = Program()
        blk = p.global_block()
        mapping: Dict[int, Variable] = {}
        for name, v in self.global_block().vars.items():
            nv = copy.copy(v)
            nv.block = blk
            nv.op = None
            blk.vars[name] = nv
            mapping[id(v)] = nv
        for op in self.global_block().ops:
            if for_test and op.attrs.get("op_role"):
                continue  # transpiler-inserted gradient / update sync
            ins = {k: [mapping[id(v)] for v in vs] for k, vs in op.inputs.items()}
            outs = {k: [mapping[id(v)] for v in vs] for k, vs in op.outputs.items()}
            attrs = dict(op.attrs)
            if for_test and "is_test" in attrs:
                attrs["is_test"] = True
            blk.append_op(op.type, ins, outs, attrs)
        p.random_seed = self.random_seed
        p._is_test = for_test
        if not for_test:
            p._optimize = self._optimize
            p._collective = self._collective
            p._pipeline_opt = self._pipeline_opt
        p._version = self._version
        return p

    def to_string(self, throw_on_error=False, with_details=False) -> str:
        lines = [repr(v) for v in self.global_block().vars.values()]
        lines += [repr(op) for op in self.global_block().ops]
        return "\n".join(lines)

    def __str__(self):
        return self.to_string()

    def _prune(self, targets):
        return self


_main_program = Program()
_startup_program = Program()


def default_main_program() -> Program:
    return _main_program


def default_startup_program() -> Program:
    return _startup_program


def switch_main_program(p: Program) -> Program:
    global _main_program
    prev, _main_program = _main_program, p
    return prev


def switch_startup_program(p: Program) -> Program:
    global _startup_program
    prev, _startup_program = _startup_program, p
    return prev


@contextlib.contextmanager
def program_guard(main_program: Program, startup_program: Optional[Program] = None):
    pm = switch_main_program(main_program)
    ps = switch_startup_program(startup_program) if startup_program is not None else None
    try:
        yield
    finally:
        switch_main_program(pm)
        if ps is not None:
            switch_startup_program(ps)


# ----------------------------------------------------------------- scope / tensors
class LoDTensor:
    """Host/device tensor + level-1 LoD (offsets).  Mirrors the parts of
    ``core.LoDTensor`` scripts use: ``set``, ``lod``/``set_lod``,
    ``recursive_sequence_lengths``, ``np.array(t)``, ``shape()``."""

    def __init__(self, value: Optional[torch.Tensor] = None, lod: Optional[List[List[int]]] = None):
        self.value = value
        self._lod = lod or []

    def set(self, arr, place=None):
        dev = to_device(place) if place is not None else (self.value.device if self.value is not None
                                                          else torch.device("cpu"))
        t = torch.as_tensor(np.asarray(arr))
        if self.value is not None and self.value.shape == t.shape:
            self.value.copy_(t.to(self.value.dtype))
        else:
            self.value = t.to(dev)

    def lod(self):
        return self._lod

    def set_lod(self, lod):
        self._lod = [list(map(int, l)) for l in lod]

    def set_recursive_sequence_lengths(self, lens):
        out = []
        for level in lens:
            offs = [0]
            for n in level:
                offs.append(offs[-1] + int(n))
            out.append(offs)
        self._lod = out

    def recursive_sequence_lengths(self):
        return [[b - a for a, b in zip(l[:-1], l[1:])] for l in self._lod]

    def shape(self):
        return list(self.value.shape) if self.value is not None else []

    def __array__(self, dtype=None, copy=None):
        a = self.value.detach().float().cpu().numpy() if self.value.dtype == torch.bfloat16 \
            else self.value.detach().cpu().numpy()
        return a.astype(dtype) if dtype is not None else a

    def numpy(self):
        return self.__array__()


def create_lod_tensor(data, recursive_seq_lens, place=None) -> LoDTensor:
    if isinstance(data, list):
        data = np.concatenate([np.asarray(d).reshape(len(d), -1) for d in data], 0)
    t = LoDTensor()
    t.set(np.asarray(data), place)
    t.set_recursive_sequence_lengths(recursive_seq_lens)
    return t


class _ScopeVar:
    def __init__(self, scope: "Scope", name: str):
        self.scope, self.name = scope, name

    def get_tensor(self) -> LoDTensor:
        t = self.scope._tensors.get(self.name)
        return LoDTensor(t)

    def set_value(self, arr):
        self.scope.set(self.name, torch.as_tensor(np.asarray(arr)))


class Scope:
    """name -> torch.Tensor store for persistable variables (params,
    data_norm summaries, optimizer moments)."""

    def __init__(self):
        self._tensors: Dict[str, torch.Tensor] = {}

    def var(self, name: str) -> _ScopeVar:
        return _ScopeVar(self, name)

    def find_var(self, name: str) -> Optional[_ScopeVar]:
        return _ScopeVar(self, name) if name in self._tensors else None

    def get(self, name: str) -> torch.Tensor:
        return self._tensors[name]

    def set(self, name: str, t: torch.Tensor):
        old = self._tensors.get(name)
        if old is not None and old.shape == t.shape:
            with torch.no_grad():
                old.copy_(t.to(old.device, old.dtype))
        else:
            self._tensors[name] = t

    def __contains__(self, name):
        return name in self._tensors

    def names(self) -> List[str]:
        return list(self._tensors)

    def drop_kids(self):
        pass


_global_scope = Scope()


def global_scope() -> Scope:
    return _global_scope


@contextlib.contextmanager
def scope_guard(scope: Scope):
    global _global_scope
    prev, _global_scope = _global_scope, scope
    try:
        yield
    finally:
        _global_scope = prev


def in_dygraph_mode() -> bool:
    return False
