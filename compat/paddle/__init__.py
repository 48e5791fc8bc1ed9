"""Opt-in alias package so unmodified PaddleBox scripts run on this engine:
with ``compat/`` on ``PYTHONPATH``, ``import paddle.fluid as fluid`` and
``from paddle.distributed import fleet`` resolve to ``paddlebox_amd.fluid`` /
``paddlebox_amd.fleet``.  Only the PaddleBox training surface is provided
(SURVEY §7.2.4)."""
import sys as _sys

from paddlebox_amd import fleet as _fleet_mod
from paddlebox_amd import fluid  # noqa: F401
from paddlebox_amd.fluid import dataset as _dataset
from paddlebox_amd.utils import flags as _flags

_sys.modules.setdefault("paddle.fluid", fluid)
_sys.modules.setdefault("paddle.fluid.core", fluid.core)
_sys.modules.setdefault("paddle.fluid.layers", fluid.layers)
_sys.modules.setdefault("paddle.fluid.contrib", fluid.contrib)
_sys.modules.setdefault("paddle.fluid.dataset", _dataset)
_sys.modules.setdefault("paddle.fluid.transpiler", fluid.transpiler)


class _Distributed:
    fleet = _fleet_mod


distributed = _Distributed()
_sys.modules.setdefault("paddle.distributed", distributed)
_sys.modules.setdefault("paddle.distributed.fleet", _fleet_mod)


def enable_static():
    """Static graph is the only mode of the fluid front end."""


set_flags = _flags.set_flags
get_flags = _flags.get_flags
