"""LayerHelper: what every ``fluid.layers`` function uses to create
parameters (main-program Parameter + startup-program ``init_param`` op),
temporaries and ops (reference ``py/fluid/layer_helper.py``)."""
from __future__ import annotations

from typing import Optional, Sequence

from . import initializer as I
from .framework import (Parameter, ParamAttr, Variable, default_main_program, default_startup_program,
                        unique_name)


class LayerHelper:
    def __init__(self, layer_type: str, name: Optional[str] = None):
        self.layer_type = layer_type
        self.name = name or unique_name.generate(layer_type)

    @property
    def main_program(self):
        return default_main_program()

    @property
    def startup_program(self):
        return default_startup_program()

    @property
    def block(self):
        return self.main_program.global_block()

    def create_parameter(self, attr, shape: Sequence[int], dtype="float32", default_initializer=None,
                         is_bias: bool = False, suffix: str = "w") -> Optional[Parameter]:
        attr = ParamAttr._to_attr(attr)
        if attr is None:
            return None
        name = attr.name or unique_name.generate(f"{self.name}.{'b' if is_bias else suffix}")
        init = attr.initializer or default_initializer or (I.Constant(0.0) if is_bias else I.Xavier())
        p = self.block.create_parameter(name, shape, dtype, initializer=init, trainable=attr.trainable,
                                        learning_rate=attr.learning_rate, regularizer=attr.regularizer,
                                        need_clip=attr.need_clip)
        sb = self.startup_program.global_block()
        if not sb.has_var(name):
            sv = sb.create_parameter(name, shape, dtype, initializer=init, trainable=attr.trainable,
                                     learning_rate=attr.learning_rate)
            sb.append_op("init_param", outputs={"Out": [sv]}, attrs={"initializer": init})
        return p

    def create_variable_for_type_inference(self, dtype="float32", shape=(), lod_level=0,
                                           stop_gradient=False) -> Variable:
        return self.block.create_var(unique_name.generate(f"{self.name}.tmp"), shape, dtype, lod_level,
                                     stop_gradient=stop_gradient)

    def create_global_variable(self, name=None, shape=(), dtype="float32", persistable=True, value=0.0):
        name = name or unique_name.generate(f"{self.name}.global")
        v = self.block.create_var(name, shape, dtype, persistable=persistable, stop_gradient=True)
        sb = self.startup_program.global_block()
        if not sb.has_var(name):
            sv = sb.create_var(name, shape, dtype, persistable=True)
            sb.append_op("init_param", outputs={"Out": [sv]}, attrs={"initializer": I.Constant(value)})
        return v

    def append_op(self, type, inputs=None, outputs=None, attrs=None):  # noqa: A002
        return self.block.append_op(type, inputs, outputs, attrs)

    def append_activation(self, x: Variable, act: Optional[str]) -> Variable:
        if not act:
            return x
        out = self.create_variable_for_type_inference(x.dtype, x.shape, x.lod_level)
        self.append_op(act, {"X": [x]}, {"Out": [out]})
        return out
